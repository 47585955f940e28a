#!/bin/bash
# Round 4: k_small_cg with branch-free row loops -- phases, tests, theta timings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04k; mkdir -p $O
LRS_SMALL_CG=1 timeout -k 10 200 python3 -u scripts/small_phase.py theta3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
timeout -k 10 400 python3 -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_small_cg.py tests/test_capi.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.txt | tail -8
[ $rc -le 1 ] || exit $rc
for v in 1 0; do
  for t in theta3 theta3x3; do
    LRS_SMALL_CG=$v timeout -k 10 120 python3 -u scripts/admm_probe.py $t >> $O/theta.txt 2>&1 || { tail -5 $O/theta.txt; exit 1; }
  done
  echo "LRS_SMALL_CG=$v done" >> $O/theta.txt
done
cat $O/theta.txt
# headline factor layout A/B (G67, r = 19: default 8 lanes x 3 doubles, ld 24)
H="--no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded"
for v in default 8x4 16x2 default 8x4; do
  if [ $v = default ]; then unset LRS_LAYOUT; else export LRS_LAYOUT=$v; fi
  timeout -k 10 200 python3 -u bench.py --steps 3000 --warmup 300 $H > $O/head_$v.log 2>&1 || { tail -5 $O/head_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('LRS_LAYOUT=$v', round(d['value']), [round(s['avg_launch_us'], 2) for s in d['roofline']['stages']])" $O/head_$v.log | tee -a $O/head.txt
done
unset LRS_LAYOUT
exit $rc
