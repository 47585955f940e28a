#!/bin/bash
# bench.py's sharded legs (G81, C5, 2000^2 torus) on a forced one-rank RCCL shard, a fresh id per leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03z; mkdir -p $O
LRS_FORCE_SHARD=1 timeout -k 10 500 python3 -u bench.py --steps 50 --warmup 5 --no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --sharded-all > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['sharded']; print(json.dumps({k: s[k] for k in s if k not in ('c5','torus2000')})); print(json.dumps(s.get('c5'))); print(json.dumps(s.get('torus2000')))" $O/bench.log
echo done
