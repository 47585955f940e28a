#!/bin/bash
# GPU box: column-tiled long-row kernels -- parity (dense-objective and steps tests, path 3
# included), then C5 / C5b at full size.
set -e
mkdir -p gpurun_out/tile
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_densec.py tests/test_gpu_steps.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tile/tests.log 2>&1 || { tail -40 gpurun_out/tile/tests.log; exit 1; }
tail -2 gpurun_out/tile/tests.log
timeout -k 10 600 python3 -u scripts/c5_probe.py 10000 1000000 128 20 > gpurun_out/tile/c5.log 2>&1
cat gpurun_out/tile/c5.log
timeout -k 10 600 python3 -u scripts/c5b_probe.py 10000 1000000 128 20 > gpurun_out/tile/c5b.log 2>&1
cat gpurun_out/tile/c5b.log
