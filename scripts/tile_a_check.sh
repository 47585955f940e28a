#!/bin/bash
# GPU box: stage A's lower pattern in 2-D LDS tiles (k_tile_a) and the tiled A(X Y^T) --
# per-trip parity on every golden instance, then C5 with the stage-A tiles off and on.
set -e
mkdir -p gpurun_out/ta
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_steps.py tests/test_gpu_auv_tiles.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ta/tests.log 2>&1 || { tail -40 gpurun_out/ta/tests.log; exit 1; }
tail -3 gpurun_out/ta/tests.log
LRS_SLOT_TILES=0 timeout -k 10 600 python3 -u scripts/c5_probe.py 10000 1000000 128 30 > gpurun_out/ta/c5_off.log 2>&1
cat gpurun_out/ta/c5_off.log
timeout -k 10 600 python3 -u scripts/c5_probe.py 10000 1000000 128 30 > gpurun_out/ta/c5_on.log 2>&1
cat gpurun_out/ta/c5_on.log
timeout -k 10 300 python3 -u scripts/c5_probe.py 10000 100000 128 60 > gpurun_out/ta/c5_m1e5.log 2>&1
cat gpurun_out/ta/c5_m1e5.log
O=$GRAFT_REPO_ROOT/gpurun_out/ta; R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 30 > $O/trace.log 2>&1) || exit 1
python3 - "$O/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:50].ljust(51), r['Calls'].rjust(5), '%10.1f us' % (float(r['AverageNs']) / 1e3), r['Percentage'])
PY
