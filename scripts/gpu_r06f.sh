# GPU box: k_it_b without spills -- leg profiles of the bandwidth-regime legs, then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 bash scripts/leg_profile.sh r06f g81 torus2000; echo "legs rc $?"
cat gpurun_out/r06f_g81/r06f_g81_summary.md gpurun_out/r06f_torus2000/r06f_torus2000_summary.md 2>/dev/null | grep -E "^\|" | head -40
timeout -k 10 620 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06f_pytest_gpu.txt 2>&1; echo "pytest rc $?"
tail -n 5 gpurun_out/r06f_pytest_gpu.txt
