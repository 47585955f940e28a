#!/bin/bash
# Round 4 (re-entry): headline A/B of the latency-kernel variants (one-batch argument loads,
# both-buffer speculative row loads in k_lat_b, control step on registers, partials stored by
# the control wave), the single-workgroup ADMM CG phases and theta A/B, then the whole GPU suite
# and the final-evidence script of the current build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04u; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
V="liblrsdp liblrsdp_pl liblrsdp_pin2 liblrsdp_pin2specpl liblrsdp_all4 liblrsdp_lreg liblrsdp_sreg liblrsdp_spec liblrsdp_pin liblrsdp_pinall liblrsdp_pin2spec liblrsdp_pin2pl"
for v in $V $V; do
  LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
LRS_SMALL_CG=1 timeout -k 10 300 python3 -u scripts/small_phase.py theta3 theta3x3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
for v in 1 0; do
  for t in theta3 theta3x3; do
    LRS_SMALL_CG=$v timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
  echo "LRS_SMALL_CG=$v done" >> $O/theta.txt
done
cat $O/theta.txt
bash scripts/gpu_r04t.sh
