#!/bin/bash
# sharded dense objective + auut parity, then the bench (N = 1) with a kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03h
timeout -k 10 600 python -u -m pytest -q -rfE -x --timeout 300 --timeout-method thread \
  "tests/test_gpu_densec.py::test_sharded_dense_objective_steps_match_reference" \
  "tests/test_gpu_densec.py::test_sharded_dense_objective_solve_matches_single_gpu" \
  "tests/test_gpu_parity.py::test_constraint_entry_auut_matches_pattern_path" \
  > gpurun_out/r03h/pytest.log 2>&1
rc=$?
tail -8 gpurun_out/r03h/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err
rc=$?
tail -c 3000 gpurun_out/r03h/bench.json
exit $rc
