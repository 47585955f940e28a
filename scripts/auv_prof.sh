#!/bin/bash
# GPU box: kernel trace (csv) of the C5 probe (tiled A(UU^T) split into tile / sum kernels)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/auvp; R=$GRAFT_REPO_ROOT
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 10 > $O/trace.log 2>&1) || exit 1
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -14
