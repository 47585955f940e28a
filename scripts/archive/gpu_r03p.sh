#!/bin/bash
# full GPU suite on the reworked tile kernels + exact-length batches + kernel-argument control
# upload; headline at the driver's sample size; C5 kernel traces: this build vs HEAD (_build/base)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rfE --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -8 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
NO="--no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded"
for s in 20 20 20 3000; do
  timeout -k 10 200 python3 -u bench.py --steps $s --warmup 5 $NO > $O/b_$s.log 2>&1 || { tail -5 $O/b_$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b_$s.log $s
done
for v in cur base; do
  L=""; [ $v = base ] && L=$R/ltr-lowrank-sdp_amd/_build/base/liblrsdp.so
  (cd /tmp && export TMPDIR=/tmp && LRS_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_$v.log 2>&1) || { tail -5 $O/c5_$v.log; exit 1; }
  grep -E "alm|stages" $O/c5_$v.log
done
echo done
