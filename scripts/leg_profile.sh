#!/bin/bash
# GPU box: rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of bench legs run
# alone (scripts/leg_probe.py), summarised over the timed relaunch loops only
# (scripts/leg_summary.py).  usage: leg_profile.sh <tag> <leg> [<leg> ...]
# -> gpurun_out/<tag>_<leg>/<tag>_<leg>_{summary.md,pmc.json}
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for LEG in "$@"; do
  O=$R/gpurun_out/${TAG}_${LEG}; mkdir -p $O
  P="$R/scripts/leg_probe.py $LEG 10"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -u $P > $O/trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 -u $P > $O/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 -u $P > $O/write.log 2>&1
  python3 $R/scripts/leg_summary.py $O ${TAG}_${LEG} > /dev/null
  find $O -name "*.csv" ! -name "*kernel_stats.csv" -delete
  echo "leg $LEG done"
done
