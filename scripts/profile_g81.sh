#!/bin/bash
# GPU box: the north-star workload (G81-like torus, n = 20 000, r = 64) under rocprofv3: kernel
# trace + stats (per-kernel time, VGPRs, grid), then one SQ pass and the FETCH / WRITE passes,
# summarised per kernel into gpurun_out/<tag>/ (scripts/pmc_kernels.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05g81}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="$R/scripts/g81_probe.py"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u $P 500 > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 -u $P 200 > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 -u $P 200 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 -u $P 200 > $O/write.log 2>&1 || exit 1
python3 $R/scripts/pmc_kernels.py $O > $O/summary.md
find $O -name "*.csv" ! -name "*kernel_stats.csv" -delete
cat $O/summary.md
