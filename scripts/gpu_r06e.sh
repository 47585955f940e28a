# GPU box: the driver's default bench line, then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r06e_bench.json.log 2> gpurun_out/r06e_bench.err; echo "bench rc $?"
tail -c 3000 gpurun_out/r06e_bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06e_smoke.txt 2>&1; echo "smoke rc $?"; cat gpurun_out/r06e_smoke.txt
