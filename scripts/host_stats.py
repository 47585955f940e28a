#!/usr/bin/env python3
"""Diagnostics (GPU box): host-loop statistics of the phase-1 throughput run (LRS_STATS=1)."""
import importlib
import os
import sys

os.environ["LRS_STATS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cols = int(sys.argv[2]) if len(sys.argv) > 2 else 100
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
path = bench.instance_for(0, rows, cols, cache)
sv = solver.Solver(path)
r = sv.determine_rank()[0]
kw = dict(fixedRank=r, reoptLevel=0)
sv.alm_throughput(0, 300, **kw)
out = sv.alm_throughput(0, 2000, **kw)
print(f"rank={r}: {out['done'] / out['seconds']:.1f} it/s ({out['seconds'] * 1e6 / out['done']:.1f} us/it)", flush=True)
res = sv.solve(reoptLevel=0, heuristicFactor=10.0, phase1Tol=1e-2)
print("gset-flags solve:", {k: res[k] for k in ("solve_time", "alm_inner", "admm_iter", "pobj")}, flush=True)
