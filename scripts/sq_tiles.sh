#!/bin/bash
# GPU box: SQ counters (two passes) over the C5 probe for the 2-D tile kernels.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sqt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/p2.log 2>&1
for p in p1 p2; do
  f=$(ls $O/$p/*counter_collection.csv | head -1)
  for c in $(python3 -c "import csv,sys; print(' '.join(sorted({r['Counter_Name'] for r in csv.DictReader(open(sys.argv[1]))})))" $f); do
    for k in k_tile_a k_tile_b1 k_tile_b2 k_auv_tile; do
      python3 $R/scripts/pmc_sum.py $f $c $k >> $O/out.txt
    done
  done
done
find $O -name "*.csv" -delete
cat $O/out.txt
