#!/bin/bash
# GPU box: A(X Y^T) over 2-D LDS tiles -- parity (tiled vs reference golden / gather), then
# C5 at full size with the tiles off and on, then a kernel trace of the tiled C5 probe.
set -e
mkdir -p gpurun_out/auv
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_auv_tiles.py -x -v --timeout 300 --timeout-method thread > gpurun_out/auv/tests.log 2>&1 || { tail -40 gpurun_out/auv/tests.log; exit 1; }
tail -3 gpurun_out/auv/tests.log
LRS_AUV_TILES=0 timeout -k 10 600 python3 -u scripts/c5_probe.py 10000 1000000 128 10 > gpurun_out/auv/c5_gather.log 2>&1
cat gpurun_out/auv/c5_gather.log
timeout -k 10 600 python3 -u scripts/c5_probe.py 10000 1000000 128 10 > gpurun_out/auv/c5_tiles.log 2>&1
cat gpurun_out/auv/c5_tiles.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/auv/prof -o c5 -- python3 -u scripts/c5_probe.py 10000 1000000 128 10 > gpurun_out/auv/prof.log 2>&1
f=$(find gpurun_out/auv/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -14
