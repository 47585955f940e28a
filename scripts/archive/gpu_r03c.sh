#!/bin/bash
# tile-kernel LDS conflicts: parity of the swizzled tiles + C5 stage times with / without
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03c
timeout -k 10 600 python -u -m pytest -q -rfE --timeout 300 --timeout-method thread \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py "tests/test_gpu_steps.py::test_lbfgs_ring_of_one" \
  "tests/test_gpu_steps.py::test_lbfgs_ring_of_three_matches_reference" -k "not full_size" > gpurun_out/r03c/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r03c/pytest.log
[ $rc -eq 0 ] || exit $rc
for swz in 0 1; do
  LRS_TILE_SWZ=$swz timeout -k 10 300 python -u scripts/c5_probe.py 10000 1000000 128 30 > gpurun_out/r03c/c5_swz$swz.log 2>&1 || exit $?
  echo "swz=$swz"; cat gpurun_out/r03c/c5_swz$swz.log
done
