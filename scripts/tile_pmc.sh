#!/bin/bash
# GPU box: C5 stage kernels with and without column tiles: time and FETCH_SIZE per dispatch.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tilepmc
mkdir -p $O
: > $O/out.txt
for t in tiles untiled; do
  if [ $t = untiled ]; then export LRS_NO_TILES=1; fi
  echo "== $t" >> $O/out.txt
  timeout -k 10 300 python3 -u $R/scripts/c5_probe.py 10000 1000000 128 20 >> $O/out.txt 2>&1
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$t -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/$t.log 2>&1)
  python3 $R/scripts/pmc_sum.py $(ls $O/$t/*counter_collection.csv | head -1) FETCH_SIZE k_ >> $O/out.txt
  find $O/$t -name "*.csv" -delete
done
cat $O/out.txt
