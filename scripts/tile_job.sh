set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05s
timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 20 > gpurun_out/r05s/c5.txt 2>&1 || exit $?
grep -E "alm|stages|auut" gpurun_out/r05s/c5.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5_steps.py tests/test_gpu_shard_tiles.py tests/test_gpu_auv_tiles.py tests/test_gpu_steps.py > gpurun_out/r05s/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r05s/pytest.txt; exit $rc
