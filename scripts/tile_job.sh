set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/${TAG:-r05s}; mkdir -p $O
timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 20 > $O/c5.txt 2>&1 || exit $?
grep -E "alm|stages|auut" $O/c5.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5_steps.py tests/test_gpu_shard_tiles.py tests/test_gpu_auv_tiles.py tests/test_gpu_steps.py > $O/pytest.txt 2>&1; rc=$?; tail -3 $O/pytest.txt; exit $rc
