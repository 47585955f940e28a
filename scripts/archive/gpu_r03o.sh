#!/bin/bash
# tile kernels reworked (k_tile_a at 1024 threads, k_tile_b2 16 lanes a row over entry-ordered S,
# k_tile_b1 epilogue loads batched): parity suites, then C5 timings and a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_steps.py tests/test_gpu_densec.py > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_1024.log 2>&1 || { tail -5 $O/c5_1024.log; exit 1; }
cat $O/c5_1024.log
LRS_TILE_A_NT=512 timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_512.log 2>&1 || { tail -5 $O/c5_512.log; exit 1; }
cat $O/c5_512.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/trace.log 2>&1) || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
head -25 $f
