#!/bin/bash
# Round 4: latency blocks sized at run time (row waves per block chosen so the grid fills the
# CUs) vs the fixed 7 row waves (LRS_LAT_ROWWAVES=7), 16-byte row loads (x4 variants), then the
# GPU suite and the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04w; mkdir -p $O
B=$R/ltr-lowrank-sdp_amd/_build
for rep in 1 2 3; do
  for v in auto w7 w5 x4; do
    case $v in
      auto) LIB=liblrsdp; W= ;; w7) LIB=liblrsdp; W=7 ;; w5) LIB=liblrsdp; W=5 ;; *) LIB=liblrsdp_$v; W= ;;
    esac
    echo -n "$v: " >> $O/ab.txt
    LRS_LAT_ROWWAVES=$W LRS_VAR_PATHS=0 timeout -k 10 120 python3 -u scripts/variants.py $B/$LIB.so >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
timeout -k 10 900 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests > $O/pytest.txt 2>&1
rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --gpus 1 > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'), [ (r['config'], r.get('speedup')) for r in d.get('configs_wall_clock_to_eps', [])])" $O/bench.json.log
