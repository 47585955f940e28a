# GPU box: bandwidth-regime unroll variants A/B, then the tests touched by the XWG fallback
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bw_variants_ab.py main bwu2 bwu4 bwub2 bwub4 > gpurun_out/r06d_bw_ab.txt 2>&1; echo "ab rc $?"
cat gpurun_out/r06d_bw_ab.txt
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_steps.py -k "single_workgroup or falls_back" > gpurun_out/r06d_pytest.txt 2>&1; echo "pytest rc $?"
grep -E "passed|failed|FAIL" gpurun_out/r06d_pytest.txt | tail -8
