# GPU box: fused-vs-split stage A test, g81 leg profile with the fused stage A, bench line, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bw_kernels.py -k fused > gpurun_out/r06n_fused.txt 2>&1; echo "fused test rc $?"
grep -E "PASS|FAIL|Error|assert" gpurun_out/r06n_fused.txt | head -20
timeout -k 10 300 bash scripts/leg_profile.sh r06n g81; echo "legs rc $?"
grep -E "^\| " gpurun_out/r06n_g81/r06n_g81_summary.md | head -12
cp gpurun_out/r06n_g81/r06n_g81_summary.md gpurun_out/r06n_g81/r06n_g81_pmc.json profiles/
cp gpurun_out/r06n_g81/trace/run_kernel_stats.csv profiles/r06n_g81_kernel_stats.csv
timeout -k 10 900 python -u bench.py > gpurun_out/r06n_bench.json.log 2> gpurun_out/r06n_bench.err; echo "bench rc $?"
tail -c 600 gpurun_out/r06n_bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06n_smoke.txt 2>&1; echo "smoke rc $?"; cat gpurun_out/r06n_smoke.txt
