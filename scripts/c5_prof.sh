#!/bin/bash
# GPU box: kernel trace of the C5 probe (scripts/c5_probe.py, 20 iterations), summarised per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r05c5}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/trace.log 2>&1 || exit 1
python3 $R/scripts/pmc_kernels.py $O > $O/summary.md
find $O -name "*.csv" ! -name "*kernel_stats.csv" -delete
head -30 $O/summary.md
