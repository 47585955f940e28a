#!/bin/bash
# One GPU-box pass: gpu tests, smoke, full bench (run from the repo root).
# Test FAILURES (pytest exit 1) still go on to smoke and bench; anything else (a crash,
# a signal, a time limit) ends the call there.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-check}
shift
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest ended with $rc"; tail -40 $O/pytest_gpu.log; exit 1; fi
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
