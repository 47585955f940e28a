#!/bin/bash
# GPU box: the at-scale instance (torus 2000^2, r = 16) and the G81-like instance with the
# XCD-chunked row order (default build) and without it (liblrsdp_noxcd.so), then FETCH_SIZE
# passes of both at scale.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-xcd}
mkdir -p $O
cd $R
for lib in "" "$R/ltr-lowrank-sdp_amd/_build/liblrsdp_noxcd.so"; do
  echo "== lib ${lib:-default}"
  LRS_LIB=$lib timeout -k 10 300 python -u scripts/scale_probe.py 2000 16 40 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for lib in "" "$R/ltr-lowrank-sdp_amd/_build/liblrsdp_noxcd.so"; do
  tag=$([ -z "$lib" ] && echo xcd || echo noxcd)
  LRS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$tag -o run -- python3 $R/scripts/scale_probe.py 2000 16 10 > $O/fetch_$tag.log 2>&1 || exit 1
  python3 - $O/fetch_$tag/run_counter_collection.csv <<'PY'
import csv, collections, sys
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"].split("(")[0][-40:]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) / len(v) > 1e5:
        print(f"  {k}: {len(v)} dispatches, FETCH_SIZE {sum(v) / len(v) / 1e6:.3f} GB-ish (KB units / 1e6)")
PY
  find $O/fetch_$tag -name "*.csv" -delete
done
