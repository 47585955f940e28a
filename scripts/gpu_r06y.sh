# GPU box: k_small_alm's dependent global loads batched / issued a slot ahead -- parity, A/B, phases
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_steps.py tests/test_gpu_configs.py tests/test_gpu_threads.py > gpurun_out/r06y_pytest.txt 2>&1; rc=$?; echo "pytest rc $rc"; tail -n 4 gpurun_out/r06y_pytest.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/small_lib_ab.py theta3 theta3x3 > gpurun_out/r06y_ab.txt 2>&1; echo "ab rc $?"; cat gpurun_out/r06y_ab.txt
timeout -k 10 120 python -u scripts/small_phase.py theta3 theta3x3 > gpurun_out/r06y_phase.txt 2>&1; echo "phase rc $?"; cat gpurun_out/r06y_phase.txt
