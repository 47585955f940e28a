#!/bin/bash
# GPU box: dense-objective tests, then the C5b probe at test and full size.
set -e
mkdir -p gpurun_out/c5b
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_densec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5b/tests.log 2>&1
timeout -k 10 300 python3 -u scripts/c5b_probe.py 2000 100000 64 20 > gpurun_out/c5b/probe.log 2>&1
timeout -k 10 600 python3 -u scripts/c5b_probe.py 10000 1000000 128 20 >> gpurun_out/c5b/probe.log 2>&1
tail -2 gpurun_out/c5b/tests.log
cat gpurun_out/c5b/probe.log
