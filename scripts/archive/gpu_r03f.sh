#!/bin/bash
# path-4 (single-workgroup) parity tests, then theta3 / theta3x3 solves: default, constant C,
# constant C + the single-workgroup inner loop
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03f
timeout -k 10 600 python -u -m pytest -q -rfE -x --timeout 120 --timeout-method thread \
  "tests/test_gpu_steps.py::test_single_workgroup_inner_loop_matches_reference" \
  "tests/test_gpu_steps.py::test_single_workgroup_solve_matches_default" \
  > gpurun_out/r03f/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r03f/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in "0 0" "1 0" "1 1"; do
  set -- $v
  LRS_CONST_C=$1 LRS_SMALL=$2 timeout -k 10 300 python -u scripts/theta_probe.py theta3 theta3x3 > gpurun_out/r03f/probe_c$1_s$2.log 2>&1 || exit $?
  echo "const_c=$1 small=$2"; cat gpurun_out/r03f/probe_c$1_s$2.log
done
