#!/bin/bash
# Round 4 final tree: smoke() and the default bench line (what the driver runs at round end).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r04final; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 600 python3 -u bench.py > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'][:12], d['roofline']['frac'], d['roofline'].get('traffic_source','')[:40], d['build']['sources_sha256_16'], d.get('config_c5',{}).get('gpu_it_s'), d.get('config_c5b',{}).get('gpu_it_s'), [ (r['config'], round(r.get('speedup'),2)) for r in d.get('configs_wall_clock_to_eps', [])])" $O/bench.json.log
