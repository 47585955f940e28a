#!/bin/bash
# kernel traces of C5 through the sharded iteration (one-rank RCCL, LRS_FORCE_SHARD=1) and unsharded
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03ab; mkdir -p $O
for v in sharded unsharded; do
  (cd /tmp && export TMPDIR=/tmp && LRS_FORCE_SHARD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/sharded_c5_probe.py $v > $O/$v.log 2>&1) || { tail -5 $O/$v.log; exit 1; }
  grep -E "info" $O/$v.log
done
echo done
