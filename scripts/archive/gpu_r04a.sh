#!/bin/bash
# Round 4, first call: the sharded-outer-tiles patch (k_g_part guard, sharded outer SDDMM / S.X on
# the tiles, unpadded k_tile_b2 LDS rows) -- parity tests, the forced one-rank sharded bench legs,
# a kernel trace of sharded C5, and the k_tile_b2 LDS counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04a; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
LRS_FORCE_SHARD=1 timeout -k 10 400 python3 -u bench.py --steps 50 --warmup 5 --no-cpu --no-eps --no-scale \
  --no-north-star --no-configs --no-c5 --no-c5b --sharded-all > $O/bench_sharded.log 2>&1 || { tail -5 $O/bench_sharded.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); s=d['sharded']; print(json.dumps({k: s[k] for k in s if k not in ('c5','torus2000')})); print(json.dumps(s.get('c5'))); print(json.dumps(s.get('torus2000')))" $O/bench_sharded.log
cd /tmp && export TMPDIR=/tmp
LRS_FORCE_SHARD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sharded -o run -- python3 $R/scripts/sharded_c5_probe.py sharded > $O/sharded.log 2>&1 || { tail -5 $O/sharded.log; exit 1; }
grep -E "info" $O/sharded.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
f=$(ls $O/p2/*counter_collection.csv | head -1)
for c in SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS; do
  for k in k_tile_a k_tile_b1 k_tile_b2 k_auv_tile; do python3 $R/scripts/pmc_sum.py $f $c $k >> $O/sq.txt; done
done
find $O/p2 -name "*.csv" -delete
cat $O/sq.txt
grep -E "c5_probe|stage|it/s" $O/p2.log | tail -5
echo done
