#!/bin/bash
# GPU-box jobs of this round, one argument each (run through gpurun from the repo root):
#   tests [pytest args]  the -m gpu suite (or the named tests), one process, per-test timeout
#   bench [bench args]   one bench.py line
#   c5probe              C5 kernel table (scripts/c5_probe.py)
# Every GPU step has its own time limit; the first failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; TAG=${TAG:-r05}; O=$R/gpurun_out/$TAG; mkdir -p $O
job=$1; shift
case $job in
tests)
    timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
        > $O/pytest.txt 2>&1; rc=$?
    tail -25 $O/pytest.txt; exit $rc ;;
bench)
    timeout -k 10 600 python3 -u bench.py "$@" > $O/bench.log 2>&1; rc=$?
    tail -3 $O/bench.log; exit $rc ;;
c5probe)
    timeout -k 10 400 python3 -u scripts/c5_probe.py "$@" > $O/c5_probe.txt 2>&1; rc=$?
    tail -40 $O/c5_probe.txt; exit $rc ;;
*) echo "unknown job $job"; exit 2 ;;
esac
