#!/usr/bin/env python3
"""GPU box: BASELINE config C5 exactly as bench.py's config_c5 times it (one phase-1 solve, 3
warmup + N timed inner iterations, alm_timed) -- run under rocprofv3 --kernel-trace for the
per-kernel split of the timed iterations, including the outer-iteration boundaries' operators."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5)))
o = sv.alm_timed(3, iters, fixedRank=128, reoptLevel=0)
print("C5 %d timed iterations: %.1f it/s (%.0f us/it), inner total %d" % (
    o["done"], o["done"] / o["seconds"], o["seconds"] / o["done"] * 1e6, o["inner"]), flush=True)
sv.close()
