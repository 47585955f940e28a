#!/bin/bash
# MFMA probe sweep (clock under load); theta3x3 whole solve under rocprofv3 (the dual
# infeasibility's Lanczos graphs included) for the committed profile
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03j; mkdir -p $O
timeout -k 10 200 python -u scripts/mfma_probe_sweep.py > $O/mfma.log 2>&1 || { cat $O/mfma.log; exit 1; }
cat $O/mfma.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t33 -o run -- python3 $R/scripts/admm_probe.py theta3x3 > $O/t33.log 2>&1)
rc=$?
echo "rocprofv3 theta3x3 rc=$rc"; tail -3 $O/t33.log
exit $rc
