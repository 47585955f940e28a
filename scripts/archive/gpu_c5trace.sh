#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/c5t; mkdir -p $O
timeout -k 10 300 python3 -u scripts/c5_timed_probe.py 20 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/scripts/c5_timed_probe.py 20 > $O/trace.log 2>&1) || exit $?
cat $O/trace.log | grep -E "it/s"
