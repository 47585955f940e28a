#!/bin/bash
# round-3 final evidence: the whole GPU suite, smoke(), the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r03v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'))" $O/bench.json.log
echo done
