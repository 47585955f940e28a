# GPU box: bitwise test of k_bw_b, then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bw_kernels.py > gpurun_out/r06k_bw.txt 2>&1; rc=$?; echo "bw rc $rc"
grep -E "PASS|FAIL|Error|assert" gpurun_out/r06k_bw.txt | head -30
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06k_pytest_gpu.txt 2>&1; echo "pytest rc $?"
tail -n 8 gpurun_out/r06k_pytest_gpu.txt
