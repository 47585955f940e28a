#!/bin/bash
# GPU box: SQ counters (one pass) over the C5 probe: where the long-row kernels' wave cycles go.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/p1.log 2>&1
for c in SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS; do
  python3 $R/scripts/pmc_sum.py $(ls $O/p1/*counter_collection.csv | head -1) $c k_wide >> $O/out.txt
  python3 $R/scripts/pmc_sum.py $(ls $O/p1/*counter_collection.csv | head -1) $c "k_it_a<64, 2, 1, 1>" >> $O/out.txt
done
find $O -name "*.csv" -delete
cat $O/out.txt
