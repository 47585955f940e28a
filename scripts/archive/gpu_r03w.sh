#!/bin/bash
# k_tile_a with the next chunk's loads in flight (LRS_TILE_A_PF=1, _build/var) against the
# default: C5 kernel traces
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03w; mkdir -p $O
for v in pf base; do
  L=$R/ltr-lowrank-sdp_amd/_build/var/liblrsdp.so; P=1; [ $v = base ] && P=0
  (cd /tmp && export TMPDIR=/tmp && LRS_LIB=$L LRS_TILE_A_PF=$P timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_$v.log 2>&1) || { tail -5 $O/c5_$v.log; exit 1; }
  grep -E "alm|stages" $O/c5_$v.log
done
echo done
