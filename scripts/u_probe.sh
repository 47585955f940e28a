#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in "" u2 u4; do
  lib=$([ -z "$v" ] && echo "" || echo "$R/ltr-lowrank-sdp_amd/_build/liblrsdp_$v.so")
  echo "== ${v:-u1}"
  LRS_LIB=$lib timeout -k 10 200 python -u scripts/u_probe.py || exit 1
  LRS_LIB=$lib timeout -k 10 300 python -u scripts/scale_probe.py 2000 16 40 || exit 1
done
