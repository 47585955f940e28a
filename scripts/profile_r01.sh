#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box from the repo root):
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${1:-r01}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B --steps 2000 --warmup 200 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B --steps 200 --warmup 0 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B --steps 200 --warmup 0 > $OUT/write.log 2>&1
# summarise on the box, then keep what comes back small (gpurun copies at most 64 MiB of
# gpurun_out/): only the summary and the per-kernel stats stay
mkdir -p $OUT/summary
PROF_DST=$OUT/summary python3 $R/scripts/summarize_prof.py ${1:-r01} > /dev/null
find $OUT -name "*.csv" ! -name "*_kernel_stats.csv" -delete
