#!/bin/bash
# Round 4: k_lat_a's control step on an LDS-batched register copy as the default -- headline A/B
# against the previous default (liblrsdp_prev.so), the GPU suite, the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04b4; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2 3; do
  for v in liblrsdp_prev liblrsdp; do
    LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$v.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
timeout -k 10 900 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 1 > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'), [ (r['config'], r.get('speedup')) for r in d.get('configs_wall_clock_to_eps', [])])" $O/bench.json.log
