#!/bin/bash
# Round 4: theta3 / theta3x3 ADMM with and without the single-workgroup half-step, the forced one-rank
# sharded bench legs, a kernel trace of sharded C5 and the k_tile_b2 LDS counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04b; mkdir -p $O
for v in 1 0; do
  for t in theta3 theta3x3; do
    LRS_SMALL_CG=$v timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
  echo "LRS_SMALL_CG=$v done" >> $O/theta.txt
done
cat $O/theta.txt
LRS_CG_SPLIT=1 timeout -k 10 200 python3 -u scripts/c5b_sens.py $O/c5b_s1.npz > $O/c5b_sens.txt 2>&1 || { tail -5 $O/c5b_sens.txt; exit 1; }
timeout -k 10 200 python3 -u scripts/c5b_sens.py $O/c5b_sa.npz $O/c5b_s1.npz >> $O/c5b_sens.txt 2>&1 || { tail -5 $O/c5b_sens.txt; exit 1; }
LRS_CG_SPLIT=3 timeout -k 10 200 python3 -u scripts/c5b_sens.py $O/c5b_s3.npz $O/c5b_sa.npz >> $O/c5b_sens.txt 2>&1 || { tail -5 $O/c5b_sens.txt; exit 1; }
rm -f $O/*.npz
cat $O/c5b_sens.txt
timeout -k 10 300 python3 -u scripts/c5_rate.py > $O/c5_rate.txt 2>&1 || { tail -5 $O/c5_rate.txt; exit 1; }
LRS_TILE_GLDS=1 timeout -k 10 300 python3 -u scripts/c5_rate.py >> $O/c5_rate.txt 2>&1 || { tail -5 $O/c5_rate.txt; exit 1; }
for v in 0 1; do
  LRS_TILE_GLDS=$v timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 1000000 128 20 >> $O/c5_rate.txt 2>&1 || { tail -5 $O/c5_rate.txt; exit 1; }
done
cat $O/c5_rate.txt
LRS_TILE_GLDS=1 timeout -k 10 400 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_c5_steps.py > $O/pytest_glds.txt 2>&1 || { tail -20 $O/pytest_glds.txt; exit 1; }
tail -3 $O/pytest_glds.txt
echo done
