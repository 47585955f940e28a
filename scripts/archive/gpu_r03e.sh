#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
for cc in 0 1; do
  LRS_CONST_C=$cc timeout -k 10 120 python -u scripts/theta_fixed.py theta3 3000 || exit $?
  LRS_CONST_C=$cc timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03e/prof_c$cc -o run -- python3 scripts/theta_fixed.py theta3 3000 > gpurun_out/r03e/prof_c$cc.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -q -rfE --timeout 300 --timeout-method thread tests/test_gpu_auv_tiles.py \
  "tests/test_gpu_densec.py" > gpurun_out/r03e/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r03e/pytest.log
exit $rc
