#!/bin/bash
# GPU box: Gram timings for the in-tree build, then the same under rocprofv3 for the k_gram /
# k_gram_fin split.
set -e
mkdir -p gpurun_out/gram
timeout -k 10 300 python3 -u scripts/gram_probe.py 100 19,64,128,256 > gpurun_out/gram/probe.log 2>&1
timeout -k 10 120 python3 -u scripts/gram_probe.py 316 128 >> gpurun_out/gram/probe.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/gram/prof -o run -- python3 -u $GRAFT_REPO_ROOT/scripts/gram_probe.py 100 128 > $GRAFT_REPO_ROOT/gpurun_out/gram/prof.log 2>&1
cat $GRAFT_REPO_ROOT/gpurun_out/gram/probe.log
