#!/bin/bash
# Round 4: k_small_alm's single-slot constraint phase in batches of four slots a thread
# (records, then b: one memory trip each per batch) vs the default, theta3 solves.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04cb; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2 3; do
  for v in liblrsdp liblrsdp_cb; do
    echo -n "$v: " >> $O/theta.txt
    LRS_PROBE_LIB=$B/$v.so timeout -k 10 120 python3 -u scripts/admm_probe.py theta3 >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
done
cat $O/theta.txt
