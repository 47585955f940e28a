#!/usr/bin/env python3
"""GPU box: cost of the final dual-infeasibility evaluation (device Lanczos) against the whole
solve, on the bench's G67-like instance and the bundled G11."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
for path in (bench.instance_for(0, 100, 100, cache), os.path.join(ROOT, "data", "bundled", "G11.dat-s")):
    sv = solver.Solver(path)
    for rep in range(2):
        t0 = time.perf_counter()
        r = sv.solve(reoptLevel=0, heuristicFactor=10.0, phase1Tol=1e-2)
        t1 = time.perf_counter()
        l1, lm = sv.dual_infeasibility()
        t2 = time.perf_counter()
        print(os.path.basename(path), "solve %.1f ms (alm %.1f admm %.1f) dinf call %.1f ms; dinf %.3e lam_min %s" % (
            (t1 - t0) * 1e3, r["alm_time"] * 1e3, r["admm_time"] * 1e3, (t2 - t1) * 1e3, l1, lm), flush=True)
    sv.close()
