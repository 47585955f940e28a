#!/usr/bin/env python3
"""GPU box: where a theta3 (BASELINE config C3) solve spends its time: ALM vs ADMM phase,
inner/CG iteration counts, the fixed-rank ALM iteration rate and the kernel path taken."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
for name in sys.argv[1:] or ["theta3"]:
    pth = inst.config_instance(name, cache)
    sv = solver.Solver(pth)
    t0 = time.perf_counter()
    r = sv.solve(**sdplib)
    t1 = time.perf_counter()
    print(name, "dims", sv.dims, "m", sv.m, "solve %.3f s: alm %.3f s (%d inner, %d outer) admm %.3f s (%d iter, %d cg) "
          "rank %d path %d" % (t1 - t0, r["alm_time"], r["alm_inner"], r["alm_outer"], r["admm_time"], r["admm_iter"],
                               r["cg_iter"], r["final_rank"], sv.kernel_path()), flush=True)
    rk = r["final_rank"]
    sv.alm_throughput(0, 200, fixedRank=rk, reoptLevel=0)
    o = sv.alm_throughput(0, 2000, fixedRank=rk, reoptLevel=0)
    print("  fixed-rank %d ALM: %.1f it/s (%.1f us/it), path %d" % (rk, o["done"] / o["seconds"],
                                                                   o["seconds"] / max(1, o["done"]) * 1e6,
                                                                   sv.kernel_path()), flush=True)
    ms = sv.time_stages(200)
    print("  stages (A, G, B) us per launch:", [round(x * 1e3, 2) for x in ms], flush=True)
    sv.close()
