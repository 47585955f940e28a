#!/bin/bash
# Round 4: transposed-butterfly dots in the single-workgroup kernels as the default -- its phases (diagnostics build), the GPU
# suite, the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04b3; mkdir -p $O
LRS_SMALL_CG=1 timeout -k 10 300 python3 -u scripts/small_phase.py theta3 theta3x3 > $O/small_phase.txt 2>&1 || { tail -5 $O/small_phase.txt; exit 1; }
cat $O/small_phase.txt
timeout -k 10 900 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 1 > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'), [ (r['config'], r.get('speedup')) for r in d.get('configs_wall_clock_to_eps', [])])" $O/bench.json.log
