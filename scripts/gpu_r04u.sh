#!/bin/bash
# Round 4 (re-entry): headline A/B of the latency-kernel variants (speculative both-buffer
# row loads in k_lat_b, scalar-register control step in k_lat_a), then the whole GPU suite
# and the final-evidence script of the current build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04u; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for v in liblrsdp liblrsdp_spec liblrsdp_sreg liblrsdp_pin liblrsdp_pinspec liblrsdp_pinall liblrsdp_pin2 liblrsdp_pin2spec liblrsdp liblrsdp_spec liblrsdp_sreg liblrsdp_pin liblrsdp_pinspec liblrsdp_pinall liblrsdp_pin2 liblrsdp_pin2spec; do
  LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
bash scripts/gpu_r04t.sh
