#!/bin/bash
# rocprofv3 passes on the at-scale instance (scripts/scale_probe.py): kernel trace, then
# FETCH_SIZE and WRITE_SIZE in separate PMC passes.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_${1:-scale}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="$R/scripts/scale_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $P 2000 16 40 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $P 2000 16 10 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $P 2000 16 10 > $OUT/write.log 2>&1
