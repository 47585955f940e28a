#!/bin/bash
# round-3 check: dual infeasibility (thick-restart Lanczos), config pins, C5 trips, sharded dinf
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03a
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dinf.py tests/test_gpu_configs.py tests/test_gpu_c5_steps.py \
  "tests/test_gpu_parity.py::test_dual_infeasibility_matches_dense_eig" \
  "tests/test_gpu_parity.py::test_dinf_step_cap_flagged" \
  tests/test_gpu_shard.py "tests/test_bundled.py::test_bundled_theta102_matches_reference" \
  > gpurun_out/r03a/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/r03a/pytest.log
exit $rc
