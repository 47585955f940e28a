#!/bin/bash
# Round 4: latency-kernel block size A/B (LRS_LAT_NT: 512 = 7 row waves + control wave, 448, 384
# threads -- more blocks over the 256 CUs, fewer row waves' vector memory instructions per CU),
# with the LDS-batched register control step, on the G67 headline path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04v; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
V="liblrsdp liblrsdp_base2 liblrsdp_lat7 liblrsdp_lat6 liblrsdp_lat6lreg liblrsdp_lreg liblrsdp_x4 liblrsdp_lat6x4"
for v in $V $V $V; do
  LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
done
cat $O/ab.txt
