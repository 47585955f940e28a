#!/bin/bash
# single-pass stage B over the tiles (k_tile_bx): tile / C5 / steps / shard parity, then C5
# kernel traces with k_tile_bx and with LRS_TILE_BX=0 (k_tile_b1 + k_tile_b2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03u; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_steps.py > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in bx b12; do
  E=1; [ $v = b12 ] && E=0
  (cd /tmp && export TMPDIR=/tmp && LRS_TILE_BX=$E timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_$v.log 2>&1) || { tail -5 $O/c5_$v.log; exit 1; }
  grep -E "alm|stages" $O/c5_$v.log
done
echo done
