#!/bin/bash
# GPU box: dense-objective and cone-count tests, then the C5b probe (slot vs dense path at
# n = 500 / 2000, full size dense).
set -e
mkdir -p gpurun_out/c5b
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_densec.py tests/test_gpu_parity.py -k "dense or cones" -x -q --timeout 300 --timeout-method thread > gpurun_out/c5b/tests.log 2>&1
: > gpurun_out/c5b/probe.log
for n in 500 2000; do
  for mode in 0 1; do
    echo "== n=$n LRS_DENSE_C=$mode" >> gpurun_out/c5b/probe.log
    LRS_DENSE_C=$mode timeout -k 10 300 python3 -u scripts/c5b_probe.py $n $((n * 50)) 64 20 >> gpurun_out/c5b/probe.log 2>&1
  done
done
echo "== n=10000 auto" >> gpurun_out/c5b/probe.log
timeout -k 10 600 python3 -u scripts/c5b_probe.py 10000 1000000 128 20 >> gpurun_out/c5b/probe.log 2>&1
tail -2 gpurun_out/c5b/tests.log
cat gpurun_out/c5b/probe.log
