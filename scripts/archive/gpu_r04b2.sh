#!/bin/bash
# Round 4: transposed-butterfly reductions (LRS_BFLY: the latency kernels' block partials, the
# single-workgroup CG's slot products, the single-workgroup ALM's row dots) vs the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04b2; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2 3; do
  for v in liblrsdp liblrsdp_bfly; do
    LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
for rep in 1 2; do
  for v in liblrsdp liblrsdp_bfly; do
    for t in theta3 theta3x3; do
      echo -n "$v: " >> $O/theta.txt
      LRS_PROBE_LIB=$B/$v.so timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
    done
  done
done
cat $O/theta.txt
