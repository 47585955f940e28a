#!/bin/bash
# headline at the driver's sample size (20 / 5) vs 3000 steps, a kernel + copy trace of the
# 20-step run (the fixed costs around the timed region), SQ counters of the C5 tile kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03m; mkdir -p $O
NO="--no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded"
for s in 20 20 20 3000; do
  timeout -k 10 200 python3 -u bench.py --steps $s --warmup 5 $NO > $O/b_$s.log 2>&1 || { tail -5 $O/b_$s.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b_$s.log $s
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 20 --warmup 5 $NO > $O/tr.log 2>&1) || { tail -5 $O/tr.log; exit 1; }
bash scripts/sq_tiles.sh > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
cp gpurun_out/sqt/out.txt $O/sq_tiles.txt
echo done
