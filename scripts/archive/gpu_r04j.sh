#!/bin/bash
# Round 4: k_small_cg's operator passes (diagnostics build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04j; mkdir -p $O
LRS_SMALL_CG=1 timeout -k 10 200 python3 -u scripts/small_phase.py theta3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
