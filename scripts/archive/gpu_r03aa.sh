#!/bin/bash
# final-build counters of the C5 tile kernels: SQ passes (scripts/sq_tiles.sh) and FETCH_SIZE /
# WRITE_SIZE passes over the C5 probe, per-dispatch averages per kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03aa; mkdir -p $O
bash scripts/sq_tiles.sh > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
cp gpurun_out/sqt/out.txt $O/sq_tiles.txt
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 -u $R/scripts/c5_probe.py 10000 1000000 128 4 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
  f=$(ls $O/$c/*counter_collection.csv | head -1)
  for k in k_tile_a k_tile_b1 k_tile_b2 k_auv_tile k_it_g k_it_a k_wide_bf; do python3 $R/scripts/pmc_sum.py $f $c $k >> $O/bytes.txt; done
  find $O/$c -name "*.csv" -delete
done
cat $O/bytes.txt
echo done
