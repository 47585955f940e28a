#!/bin/bash
# GPU box: dense-objective tests (latency kernels included), then theta3 / theta3x3 with the
# objective in the slots (LRS_DENSE_C=0) and on the matrix cores (LRS_DENSE_C=1).
set -e
mkdir -p gpurun_out/thd
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_densec.py -x -q --timeout 300 --timeout-method thread > gpurun_out/thd/tests.log 2>&1 || { tail -40 gpurun_out/thd/tests.log; exit 1; }
tail -2 gpurun_out/thd/tests.log
: > gpurun_out/thd/probe.log
for mode in 0 1; do
  echo "== LRS_DENSE_C=$mode" >> gpurun_out/thd/probe.log
  LRS_DENSE_C=$mode timeout -k 10 300 python3 -u scripts/theta_probe.py theta3 theta3x3 >> gpurun_out/thd/probe.log 2>&1
done
cat gpurun_out/thd/probe.log
