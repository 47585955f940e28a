#!/bin/bash
# GPU box: Gram parity tests, Gram timings, and the default bench line.
set -e
mkdir -p gpurun_out/gram
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k gram -x -q --timeout 120 --timeout-method thread > gpurun_out/gram/tests.log 2>&1
timeout -k 10 120 python3 -u scripts/gram_probe.py 100 19,64,128,256,512 > gpurun_out/gram/probe.log 2>&1
timeout -k 10 120 python3 -u scripts/gram_probe.py 316 64,128,256 >> gpurun_out/gram/probe.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/gram/bench.log 2>&1
tail -2 gpurun_out/gram/tests.log
cat gpurun_out/gram/probe.log
