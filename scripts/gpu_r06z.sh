# GPU box: the round's final library -- GPU suite, smoke, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r06z_pytest_gpu.txt 2>&1; echo "pytest rc $?"
tail -n 4 gpurun_out/r06z_pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z_smoke.txt 2>&1; echo "smoke rc $?"; cat gpurun_out/r06z_smoke.txt
timeout -k 10 900 python -u bench.py > gpurun_out/r06z_bench.json.log 2> gpurun_out/r06z_bench.err; echo "bench rc $?"
