#!/bin/bash
# r02c: the GPU suite + smoke + bench, then a rocprofv3 kernel trace of a theta3x3 solve
# (its final dual infeasibility replays the cached Lanczos graphs; r01k segfaulted there).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_check.sh r02c || exit 1
O=$R/gpurun_out/r02c/admmprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/scripts/admm_probe.py theta3x3 > $O/trace.log 2>&1
echo "admm profile rc=$?"
tail -3 $O/trace.log
find $O -name "*kernel_stats.csv" | head -3
find $O -name "*.csv" ! -name "*_kernel_stats.csv" -delete
