#!/bin/bash
# Round 4: SQ counters of the latency kernels on the G67 headline at the run-time block size
# (5 row waves a block, 250 blocks) and at the old 7 (LRS_LAT_ROWWAVES=7, 179 blocks): where the
# waves' cycles go (one --pmc pass each, 8 SQ counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04sq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
BA="$R/bench.py --no-cpu --no-eps --no-scale --no-north-star --no-configs --no-c5 --no-c5b --no-sharded --steps 300 --warmup 0"
for w in 0 7; do
  export LRS_LAT_ROWWAVES=$w
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/w$w -o run -- python3 -u $BA > $O/w$w.log 2>&1 || { tail -5 $O/w$w.log; exit 1; }
  F=$(ls $O/w$w/*counter_collection.csv | head -1)
  for c in $C; do python3 $R/scripts/pmc_sum.py $F $c k_lat_ >> $O/out_w$w.txt; done
  find $O/w$w -name "*.csv" -delete
done
unset LRS_LAT_ROWWAVES
echo "== row waves auto (5)"; cat $O/out_w0.txt
echo "== row waves 7"; cat $O/out_w7.txt
