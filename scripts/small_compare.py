#!/usr/bin/env python3
"""GPU box: whole solves and fixed-rank ALM rates of the small instances on the default kernel
path and on the single-workgroup inner loop (path 4), to set the path-4 auto rule."""
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
G = os.path.join(ROOT, "tests", "golden", "instances")
names = sys.argv[1:] or ["mc_rand200", "mc_torus12x10", "mc_rand300w", "theta40", "theta25x3", "rsparse60", "theta3"]
for name in names:
    pth = inst.config_instance(name, cache) if name == "theta3" else os.path.join(G, name + ".dat-s")
    row = [name]
    for path in (None, 4):
        sv = solver.Solver(pth)
        if path is not None:
            sv.set_kernel_path(path)
        t0 = time.perf_counter()
        r = sv.solve(reoptLevel=0)
        t1 = time.perf_counter()
        used = sv.kernel_path()
        rk = r["final_rank"]
        sv.alm_throughput(0, 100, fixedRank=rk, reoptLevel=0)
        o = sv.alm_throughput(0, 1000, fixedRank=rk, reoptLevel=0)
        row.append("path %d: solve %.3f s (alm %.3f, %d inner) %.1f us/it r%d" % (
            used, t1 - t0, r["alm_time"], r["alm_inner"], o["seconds"] / max(1, o["done"]) * 1e6, rk))
        sv.close()
    print(" | ".join(row), flush=True)
