#!/usr/bin/env python3
"""GPU box: a BASELINE theta config solved with bench.py's SDPLIB flags (argv: name, repeats);
LRS_SMALL / LRS_SMALL_CG_BATCH in the environment pick the inner loop and the ADMM half-steps."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
name = sys.argv[1] if len(sys.argv) > 1 else "theta3x3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
env = {k: os.environ.get(k, "-") for k in ("LRS_SMALL", "LRS_SMALL_CG_BATCH", "LRS_SMALL_MC", "LRS_LIB")}
for _ in range(reps):
    sv = solver.Solver(inst.config_instance(name, cache))
    r = sv.solve(**sdplib)
    path = sv.kernel_path()
    sv.close()
    print(f"{name} {env} path={path}: solve {r['solve_time']:.4f} s (alm {r['alm_time']:.4f}, admm {r['admm_time']:.4f}) "
          f"inner {r['alm_inner']} admm {r['admm_iter']} cg {r['cg_iter']} pobj {r['pobj']:.10g} gap {r['gap']:.2e} "
          f"pinf {r['pinf']:.2e}", flush=True)
