#!/bin/bash
# GPU box: kernel trace of one theta3x3 solve (scripts/theta_solve_time.py), summarised per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05ze}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u $R/scripts/theta_solve_time.py ${1:-theta3x3} 1 > $O/trace.log 2>&1 || exit 1
python3 $R/scripts/pmc_kernels.py $O > $O/summary.md
find $O -name "*.csv" ! -name "*kernel_stats.csv" -delete
head -40 $O/summary.md
