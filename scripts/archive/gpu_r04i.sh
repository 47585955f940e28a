#!/bin/bash
# Round 4: where k_small_cg's time goes (diagnostics build), the latency kernels' stamps, the
# small-CG / C-ABI sweep tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04i; mkdir -p $O
LRS_SMALL_CG=1 timeout -k 10 200 python3 -u scripts/small_phase.py theta3 theta3x3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
timeout -k 10 200 python3 -u scripts/stage_timing.py > $O/stage_timing.txt 2>&1 || { tail -5 $O/stage_timing.txt; exit 1; }
grep -E "block 0|it/s" $O/stage_timing.txt
timeout -k 10 400 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_small_cg.py tests/test_capi.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
exit $rc
