#!/bin/bash
# split-K cgemm parity, C5b dense product timing sweep, C5 bench-like kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -rfE -x --timeout 300 --timeout-method thread \
  "tests/test_gpu_densec.py::test_split_k_cgemm_per_trip_at_n2500" \
  "tests/test_gpu_densec.py::test_dense_objective_steps_match_reference" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for sp in 1 2 3 4 6 8; do
  LRS_CG_SPLIT=$sp timeout -k 10 200 python -u scripts/c5b_cgemm_probe.py > $O/cg_$sp.log 2>&1 || exit $?
  echo "S=$sp $(cat $O/cg_$sp.log | tail -1)"
done
timeout -k 10 300 python3 -u scripts/c5_timed_probe.py 20 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/scripts/c5_timed_probe.py 20 > $O/trace.log 2>&1) || exit $?
grep -E "it/s" $O/trace.log
