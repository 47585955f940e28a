#!/bin/bash
# Round 4 (re-entry): the whole GPU suite on the current build, then the final-evidence script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04t; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04s.sh
