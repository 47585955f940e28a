#!/bin/bash
# GPU box: stage-B partials folded once (LRS_FOLD) vs every stage-A block reducing them, at scale
# (2000^2 torus, r = 16) and on C5
set -e
mkdir -p gpurun_out/fold
for f in 0 1; do
  LRS_FOLD=$f timeout -k 10 300 python3 -u scripts/scale_probe.py 2000 16 60 > gpurun_out/fold/scale_$f.log 2>&1
  echo "fold=$f $(cat gpurun_out/fold/scale_$f.log)"
  LRS_FOLD=$f timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 30 > gpurun_out/fold/c5_$f.log 2>&1
  echo "fold=$f"; grep -E "it/s|stages" gpurun_out/fold/c5_$f.log
done
