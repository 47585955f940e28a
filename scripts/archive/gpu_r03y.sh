#!/bin/bash
# slots of long-row cones renumbered by constraint: tile / C5 / steps / shard / RCCL parity, C5
# kernel traces with and without (LRS_SLOT_RENUM=0), bench's sharded legs on a forced one-rank shard
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03y; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -rfE --timeout 600 --timeout-method thread tests/test_gpu_shard_tiles.py \
  tests/test_gpu_auv_tiles.py tests/test_gpu_c5_steps.py tests/test_gpu_steps.py tests/test_gpu_densec.py > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in renum rowmajor; do
  E=1; [ $v = rowmajor ] && E=0
  (cd /tmp && export TMPDIR=/tmp && LRS_SLOT_RENUM=$E timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5_$v.log 2>&1) || { tail -5 $O/c5_$v.log; exit 1; }
  grep -E "alm|stages" $O/c5_$v.log
done
LRS_FORCE_SHARD=1 timeout -k 10 400 python3 -u bench.py --steps 50 --warmup 5 --no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --sharded-all > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['sharded']; print(json.dumps({k: s[k] for k in s if k not in ('c5','torus2000')})); print(json.dumps(s.get('c5'))); print(json.dumps(s.get('torus2000')))" $O/bench.log
echo done
