#!/bin/bash
# GPU box: the headline iteration with kernel arguments forced into device memory or not
# (HIP_FORCE_DEV_KERNARG), in-kernel stamps + throughput for each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-kernarg}
mkdir -p $O
cd $R
for v in 1 0; do
  echo "== HIP_FORCE_DEV_KERNARG=$v"
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u scripts/stage_timing.py > $O/stage_$v.log 2>&1 || exit 1
  grep -E "it/s|KA phases|KB phases|KA:|KB:" $O/stage_$v.log | head -6
done
