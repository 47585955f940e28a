# GPU box: per-leg rocprof (kernel trace + FETCH/WRITE passes) of the legs the new stage-B kernel
# runs on, then the default bench line and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 bash scripts/leg_profile.sh r06l g81 torus2000 g67; echo "legs rc $?"
for l in g81 torus2000 g67; do
  grep -E "^\| (A|B|auut) \|" gpurun_out/r06l_$l/r06l_${l}_summary.md | tail -n 3
  cp gpurun_out/r06l_$l/r06l_${l}_summary.md gpurun_out/r06l_$l/r06l_${l}_pmc.json profiles/
  cp gpurun_out/r06l_$l/trace/run_kernel_stats.csv profiles/r06l_${l}_kernel_stats.csv
done
timeout -k 10 900 python -u bench.py > gpurun_out/r06l_bench.json.log 2> gpurun_out/r06l_bench.err; echo "bench rc $?"
tail -c 1500 gpurun_out/r06l_bench.err
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06l_smoke.txt 2>&1; echo "smoke rc $?"; cat gpurun_out/r06l_smoke.txt
