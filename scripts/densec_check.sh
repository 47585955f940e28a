#!/bin/bash
# GPU box: dense-objective parity tests.
mkdir -p gpurun_out/densec
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_densec.py -x -v --timeout 300 --timeout-method thread > gpurun_out/densec/tests.log 2>&1
rc=$?
tail -30 gpurun_out/densec/tests.log
exit $rc
