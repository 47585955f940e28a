# GPU box: k_small_alm rows phase in adjacency-length order -- phases, theta solves A/B, parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_steps.py tests/test_gpu_configs.py tests/test_gpu_threads.py > gpurun_out/r06x_pytest.txt 2>&1; rc=$?; echo "pytest rc $rc"; tail -n 4 gpurun_out/r06x_pytest.txt; [ $rc -eq 0 ] || exit 1
for f in 0 1; do LRS_SMALL_ROWSORT=$f timeout -k 10 120 python -u scripts/small_phase.py theta3 theta3x3 > gpurun_out/r06x_phase_$f.txt 2>&1 || exit 1; echo "rowsort $f"; cat gpurun_out/r06x_phase_$f.txt; done
timeout -k 10 300 python -u scripts/theta_rowsort_ab.py > gpurun_out/r06x_ab.txt 2>&1; echo "ab rc $?"; cat gpurun_out/r06x_ab.txt
