#!/bin/bash
# (RD, DD) records for k_it_g (uvp): tile / C5 / steps parity, then C5 kernel traces: this
# tile / C5 / steps parity, then C5 kernel traces: this build vs _build/var (k_tile_b1 without

cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03r; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_steps.py tests/test_gpu_densec.py > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in cur var; do
  L=""; [ $v = var ] && L=$R/ltr-lowrank-sdp_amd/_build/var/liblrsdp.so
  (cd /tmp && export TMPDIR=/tmp && LRS_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_$v.log 2>&1) || { tail -5 $O/c5_$v.log; exit 1; }
  grep -E "alm|stages" $O/c5_$v.log
done
echo done
