#!/usr/bin/env python3
"""GPU box: the G81-like north-star instance (torus 100 x 200, r = 64) with the library named
by LRS_LIB: fixed-rank ALM it/s and per-stage launch times."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
bench = importlib.import_module("bench")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
p81 = bench.instance_for(0, 100, 200, cache, seed0=81)
sv = solver.Solver(p81)
kw = dict(fixedRank=64, reoptLevel=0)
sv.alm_throughput(0, 100, **kw)
o = sv.alm_throughput(0, 1000, **kw)
ms = sv.time_stages(100)
print(f"G81 r=64: {o['done'] / o['seconds']:.0f} it/s, stages us {[round(x * 1e3, 2) for x in ms]}", flush=True)
