#!/bin/bash
# GPU box: dense-objective tests, then the C5b probe at full size (dense) under a kernel trace.
set -e
mkdir -p gpurun_out/c5b
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_densec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5b/tests.log 2>&1 || { tail -30 gpurun_out/c5b/tests.log; exit 1; }
tail -2 gpurun_out/c5b/tests.log
timeout -k 10 600 python3 -u scripts/c5b_probe.py 10000 1000000 128 20 > gpurun_out/c5b/probe.log 2>&1
cat gpurun_out/c5b/probe.log
