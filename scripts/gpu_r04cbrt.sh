#!/bin/bash
# Round 4: the wave line search's cube roots by cbrt instead of pow(., 1/3) (LRS_CBRT), G67 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04cbrt; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2 3; do
  for v in liblrsdp liblrsdp_cbrt; do
    LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
