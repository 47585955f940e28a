#!/bin/bash
# Round 4 final build: in-kernel stage stamps of the latency kernels (run-time block size) and
# the headline rocprofv3 trace + FETCH/WRITE passes (profile_r01.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04zz; mkdir -p $O
timeout -k 10 200 python3 -u scripts/stage_timing.py > $O/stage_timing.txt 2>&1 || { tail -5 $O/stage_timing.txt; exit 1; }
cat $O/stage_timing.txt
timeout -k 10 900 bash scripts/profile_r01.sh r04zz > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
head -12 $R/gpurun_out/prof_r04zz/summary/r04zz_summary.md
