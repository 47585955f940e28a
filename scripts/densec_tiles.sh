#!/bin/bash
# GPU box: dense-vs-slot per-trip agreement at n = 2000 with the 2-D tiles, then a C5 kernel trace
set -e
mkdir -p gpurun_out/dt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_densec.py -x -v --timeout 300 --timeout-method thread -k "per_trip" > gpurun_out/dt/tests.log 2>&1 || { tail -40 gpurun_out/dt/tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/dt/tests.log
O=$GRAFT_REPO_ROOT/gpurun_out/dt; R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 30 > $O/trace.log 2>&1) || exit 1
cat $O/trace.log | grep -E "it/s|stages|auut"
