#!/bin/bash
# evidence of this build: the whole GPU suite, the default bench line, the headline rocprofv3
# trace + FETCH/WRITE passes (profile_r01.sh), a C5 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'))" $O/bench.json.log
timeout -k 10 900 bash scripts/profile_r01.sh r03s > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5 -o run -- python3 $R/scripts/c5_probe.py 10000 1000000 128 20 > $O/c5.log 2>&1) || { tail -5 $O/c5.log; exit 1; }
grep -E "alm|stages" $O/c5.log
echo done
