#!/bin/bash
# GPU box: one workgroup per cone -- the inner loop's per-trip parity (theta25x3, forced) and the
# ADMM half-steps side by side against the sweep, then theta3 / theta3x3 solves (defaults, and
# theta3x3 with the multi-launch inner loop and cone-by-cone half-steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/${TAG:-r05u}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_small_cg.py "tests/test_gpu_steps.py::test_single_workgroup_inner_loop_matches_reference" "tests/test_gpu_steps.py::test_single_workgroup_solve_matches_default" tests/test_gpu_configs.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u scripts/theta_solve_time.py theta3x3 2 > $O/solve.txt 2>&1 || exit $?
LRS_SMALL=0 LRS_SMALL_CG_BATCH=0 timeout -k 10 120 python3 -u scripts/theta_solve_time.py theta3x3 1 >> $O/solve.txt 2>&1 || exit $?
timeout -k 10 120 python3 -u scripts/theta_solve_time.py theta3 2 >> $O/solve.txt 2>&1 || exit $?
cat $O/solve.txt
