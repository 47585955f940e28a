#!/bin/bash
# GPU box: the at-scale torus under kernel paths 0 (auto) and 3 (long-row k_wide kernels)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for p in 0 3; do
  echo "== path $p"
  LRS_PATH=$p timeout -k 10 300 python -u scripts/scale_probe.py 2000 16 40 || exit 1
done
