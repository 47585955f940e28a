#!/bin/bash
# Round-2 evidence on the GPU box: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of
# the bench headline (scripts/profile_r01.sh) and of the at-scale instance (profile_scale.sh),
# summaries into gpurun_out/prof_<tag>/summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
bash $R/scripts/profile_r01.sh $TAG || exit 1
bash $R/scripts/profile_scale.sh ${TAG}_scale || exit 1
mkdir -p $R/gpurun_out/prof_${TAG}_scale/summary
PROF_DST=$R/gpurun_out/prof_${TAG}_scale/summary python3 $R/scripts/summarize_prof.py ${TAG}_scale > /dev/null
find $R/gpurun_out/prof_${TAG}_scale -name "*.csv" ! -name "*_kernel_stats.csv" -delete
# C5b (dense objective): kernel trace of the probe at full size, k_cgemm's duration beside the
# bench's HIP-event figure
O=$R/gpurun_out/prof_${TAG}_c5b
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/c5b_probe.py 10000 1000000 128 10 > $O/trace.log 2>&1) || exit 1
find $O -name "*.csv" ! -name "*_kernel_stats.csv" -delete
ls $R/gpurun_out/prof_${TAG}/summary $R/gpurun_out/prof_${TAG}_scale/summary $O/trace
