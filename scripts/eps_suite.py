#!/usr/bin/env python3
"""Diagnostics (GPU box): wall-clock to eps = 1e-5 on the BASELINE configs, device vs the
reference CPU build (oracle/_ref), with benchmark.py's flags for each subtype."""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
bench = importlib.import_module("bench")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
GSET = {"reoptLevel": 0, "heuristicFactor": 10.0, "phase1Tol": 1e-2, "rhoMax": 5000.0}
SDPLIB = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
cases = [("G1", GSET), ("G22", GSET), ("G81", GSET), ("theta3", SDPLIB), ("theta3x3", SDPLIB)]
only = sys.argv[1:] or [c for c, _ in cases]
for name, flags in cases:
    if name not in only:
        continue
    path = inst.config_instance(name, cache)
    sv = solver.Solver(path)
    t0 = time.perf_counter()
    r = sv.solve(**flags)
    wall = time.perf_counter() - t0
    sv.close()
    cli = []
    for k, v in flags.items():
        cli += [f"--{k}", str(v)]
    ref = bench.cpu_reference_solve(path, cli, timeout=400)
    print(json.dumps({"case": name, "gpu_solve_s": r["solve_time"], "gpu_wall_s": wall, "alm_inner": r["alm_inner"],
                      "admm_iter": r["admm_iter"], "cg_iter": r["cg_iter"], "pobj": r["pobj"], "gap": r["gap"],
                      "pinf": r["pinf"], "ref": ref}), flush=True)
