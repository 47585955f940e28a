#!/usr/bin/env python3
"""Diagnostics (GPU box): headline ALM rate and per-stage launch times of one library
build (argv[1] = path to a liblrsdp variant), latency-regime path, G67-like torus."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")
solver.load_library(sys.argv[1])
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100
cols = int(sys.argv[3]) if len(sys.argv) > 3 else 100
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
path = bench.instance_for(0, rows, cols, cache)
for kp in [int(x) for x in os.environ.get("LRS_VAR_PATHS", "0,1").split(",")]:
    sv = solver.Solver(path)
    sv.set_kernel_path(kp)
    r = sv.determine_rank()[0]
    kw = dict(fixedRank=r, reoptLevel=0)
    sv.alm_throughput(0, 300, **kw)
    out = sv.alm_throughput(0, 3000, **kw)
    ms = sv.time_stages(200)
    print(f"{os.path.basename(sys.argv[1])} path={sv.kernel_path()}: {out['done'] / out['seconds']:.0f} it/s; "
          f"stage us {[round(x * 1e3, 2) for x in ms]}", flush=True)
    sv.close()
