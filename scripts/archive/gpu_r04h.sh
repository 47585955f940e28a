#!/bin/bash
# Round 4: the single-workgroup ADMM half-step on constant-objective cones (theta in the rank-one
# form): its tests, the theta configs, theta3 / theta3x3 ADMM with and without it, a theta3 trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04h; mkdir -p $O
timeout -k 10 200 python3 -u scripts/stage_timing.py > $O/stage_timing.txt 2>&1 || { tail -5 $O/stage_timing.txt; exit 1; }
grep -E "block 0|it/s" $O/stage_timing.txt
timeout -k 10 600 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_small_cg.py tests/test_capi.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -12
[ $rc -le 1 ] || exit $rc
! grep -q -E "Timeout \(>" $O/pytest.txt || { echo "a test timed out: stopping"; exit 3; }
for v in 1 0; do
  for t in theta3 theta3x3; do
    LRS_SMALL_CG=$v timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
  echo "LRS_SMALL_CG=$v done" >> $O/theta.txt
done
cat $O/theta.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t3 -o run -- python3 $R/scripts/admm_probe.py theta3 > $O/t3.log 2>&1) || { tail -5 $O/t3.log; exit 1; }
f=$(find $O/t3 -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -d, -f1-8 > $O/t3_stats.txt; cat $O/t3_stats.txt
find $O/t3 -name "*.csv" ! -name "*_kernel_stats.csv" -delete
exit $rc
