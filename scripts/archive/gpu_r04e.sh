#!/bin/bash
# Round 4: where the single-workgroup loop (theta3) and the latency kernels (G67) spend their
# time (diagnostics build), then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04e; mkdir -p $O
timeout -k 10 200 python3 -u scripts/small_phase.py theta3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
timeout -k 10 200 python3 -u scripts/stage_timing.py > $O/stage_timing.txt 2>&1 || { tail -5 $O/stage_timing.txt; exit 1; }
cat $O/stage_timing.txt
timeout -k 10 850 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.txt | head -20
tail -3 $O/pytest.txt
exit $rc
