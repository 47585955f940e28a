#!/bin/bash
# Round 4: the single-workgroup ADMM half-step (k_small_cg) at 1024 threads (LRS_SC_NT=1024:
# 64 row groups, half the rows per group) against 512, theta3 / theta3x3 solves; the
# multi-launch CG (LRS_SMALL_CG=0) beside them.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04y; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2; do
  for v in liblrsdp liblrsdp_cg1k; do
    for t in theta3 theta3x3; do
      echo -n "$v small_cg=1: " >> $O/theta.txt
      LRS_PROBE_LIB=$B/$v.so LRS_SMALL_CG=1 timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
    done
  done
  for t in theta3 theta3x3; do
    echo -n "liblrsdp small_cg=0: " >> $O/theta.txt
    LRS_SMALL_CG=0 timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
done
cat $O/theta.txt
