#!/usr/bin/env python3
"""GPU box A/B: theta3 / theta3x3 solves (SDPLIB flags, bench.py's configs leg) with the
single-workgroup rows phase in adjacency-length order (LRS_SMALL_ROWSORT=1, default) and in
row order (=0), alternating settings, three solves each; prints wall time and iteration counts."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
for name in sys.argv[1:] or ["theta3", "theta3x3"]:
    path = inst.config_instance(name, cache)
    res = {"0": [], "1": []}
    for rnd in range(3):
        for flag in ("0", "1"):
            os.environ["LRS_SMALL_ROWSORT"] = flag
            sv = solver.Solver(path)
            t0 = time.perf_counter()
            r = sv.solve(**sdplib)
            wall = time.perf_counter() - t0
            res[flag].append(wall)
            print(f"{name} rowsort {flag} round {rnd}: solve {wall:.4f} s alm {r['alm_time']:.4f} s "
                  f"({r['alm_inner']} inner) admm {r['admm_time']:.4f} s pobj {r['pobj']:.10g}", flush=True)
            sv.close()
    print(f"{name}: best rowsort 0 {min(res['0']):.4f} s, rowsort 1 {min(res['1']):.4f} s", flush=True)
