#!/bin/bash
# Round 4: latency kernels without the record loads of entries that carry no single
# constraint (LRS_LAT_SKIPREC, exec-masked instead of clamped), with and without 16-byte row loads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04x; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
V="liblrsdp liblrsdp_skip liblrsdp_skipx4"
for v in $V $V $V; do
  LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
