#!/usr/bin/env python3
"""GPU box: theta3 fixed-rank ALM iterations only (for a kernel trace): rank 26, N iterations."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
name = sys.argv[1] if len(sys.argv) > 1 else "theta3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
sv = solver.Solver(inst.config_instance(name, cache))
o = sv.alm_throughput(0, iters, fixedRank=26, reoptLevel=0)
print(name, "%.1f us/it" % (o["seconds"] / max(1, o["done"]) * 1e6), "path", sv.kernel_path(), flush=True)
sv.close()
