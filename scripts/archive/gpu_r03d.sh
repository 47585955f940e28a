#!/bin/bash
# constant objective (theta's C = -J as rank-one products) + the tile / C5 checks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03d
timeout -k 10 900 python -u -m pytest -q -rfE --timeout 300 --timeout-method thread \
  tests/test_gpu_steps.py tests/test_gpu_densec.py tests/test_gpu_configs.py tests/test_gpu_dinf.py \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_shard.py \
  "tests/test_gpu_parity.py::test_device_solve_matches_reference" "tests/test_gpu_parity.py::test_dual_infeasibility_matches_dense_eig" \
  tests/test_gpu_cli.py "tests/test_bundled.py::test_bundled_theta102_matches_reference" \
  > gpurun_out/r03d/pytest.log 2>&1
rc=$?
tail -12 gpurun_out/r03d/pytest.log
for swz in 0 1; do
  LRS_TILE_SWZ=$swz timeout -k 10 300 python -u scripts/c5_probe.py 10000 1000000 128 30 > gpurun_out/r03d/c5_swz$swz.log 2>&1 || exit $?
  echo "swz=$swz"; cat gpurun_out/r03d/c5_swz$swz.log
done
for cc in 0 1; do
  LRS_CONST_C=$cc timeout -k 10 300 python -u scripts/theta_probe.py theta3 theta3x3 > gpurun_out/r03d/theta_c$cc.log 2>&1
  echo "const_c=$cc"; cat gpurun_out/r03d/theta_c$cc.log
done
exit $rc
