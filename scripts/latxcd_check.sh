#!/bin/bash
# GPU box: default vs LRS_LAT_XCD latency kernels on the G67 headline: it/s, then FETCH_SIZE and
# WRITE_SIZE per dispatch of k_lat_a / k_lat_b (separate --pmc passes).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/latxcd
mkdir -p $O
L=$R/ltr-lowrank-sdp_amd/_build
for v in liblrsdp liblrsdp_latxcd; do
  timeout -k 10 120 python3 -u $R/scripts/latxcd_probe.py $L/$v.so 3000 >> $O/rate.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
for v in liblrsdp liblrsdp_latxcd; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${v}_$c -o run -- python3 -u $R/scripts/latxcd_probe.py $L/$v.so 200 > $O/${v}_$c.log 2>&1
    echo "== $v $c" >> $O/pmc.txt
    python3 $R/scripts/pmc_sum.py $(ls $O/${v}_$c/*counter_collection.csv | head -1) $c k_lat >> $O/pmc.txt
    find $O/${v}_$c -name "*.csv" -delete
  done
done
cat $O/rate.log $O/pmc.txt
