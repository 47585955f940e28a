# GPU box: G81 kernel-path A/B, then the whole -m gpu suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/g81_paths.py 2 > gpurun_out/r06c_g81_paths.txt 2>&1; echo "g81 rc $?"
LRS_FORCE_REGIME=small timeout -k 10 300 python -u scripts/g81_paths.py 1 > gpurun_out/r06c_g81_paths_small.txt 2>&1; echo "g81 small rc $?"
cat gpurun_out/r06c_g81_paths.txt gpurun_out/r06c_g81_paths_small.txt
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_pytest.txt 2>&1; rc=$?; echo "pytest rc $rc"
tail -5 gpurun_out/full_pytest.txt
[ $rc -eq 0 ] && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.txt 2>&1; echo "smoke rc $?"; cat gpurun_out/full_smoke.txt
