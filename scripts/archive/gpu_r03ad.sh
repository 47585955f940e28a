#!/bin/bash
# sharded long-row cones: k_g_part skipped on no-op iterations, the outer SDDMM / S X over the
# tiles; shard + tile parity, then the sharded-vs-unsharded C5 probe and the sharded bench legs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_shard.py tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_densec.py tests/test_gpu_dinf.py > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in sharded unsharded; do
  LRS_FORCE_SHARD=1 timeout -k 10 300 python3 $R/scripts/sharded_c5_probe.py $v > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  grep -E "info" $O/$v.log
done

(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5.log 2>&1) || { tail -5 $O/c5.log; exit 1; }
grep -E "alm|stages" $O/c5.log
echo done
