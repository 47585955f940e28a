#!/usr/bin/env python3
"""GPU box: one theta3x3 solve (BASELINE C3 multi-block) for a kernel trace of the ADMM phase."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
if os.environ.get("LRS_PROBE_LIB"):   # a variant build (ltr-lowrank-sdp_amd/_build/liblrsdp_<v>.so)
    solver.load_library(os.environ["LRS_PROBE_LIB"])
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
name = sys.argv[1] if len(sys.argv) > 1 else "theta3x3"
sv = solver.Solver(inst.config_instance(name, cache))
t0 = time.perf_counter()
r = sv.solve(**sdplib)
print(name, "solve %.3f s alm %.3f admm %.3f admm_iter %d cg %d" % (time.perf_counter() - t0, r["alm_time"],
                                                                   r["admm_time"], r["admm_iter"], r["cg_iter"]))
sv.close()
