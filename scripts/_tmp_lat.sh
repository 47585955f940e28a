set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lat; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  LRS_NO_LAT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o run -- python3 $R/scripts/lat_run.py > $O/run$v.log 2>&1 || exit 1
  tail -1 $O/run$v.log
done
