#!/usr/bin/env python3
"""Diagnostics (GPU box): the at-scale instance of bench.py (2000 x 2000 torus, r = 16)
alone, for rocprofv3 kernel-trace / PMC passes.  Prints the stage and A(UU^T) timings."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
side = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 16
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 40
sv = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(side, side, 2000)))
if os.environ.get("LRS_PATH"):
    sv.set_kernel_path(int(os.environ["LRS_PATH"]))
out = sv.alm_throughput(0, iters, fixedRank=rank, reoptLevel=0)
ms = sv.time_stages(5)
by = sv.stage_bytes()
am = sv.time_auut(5)
ab = sv.auut_bytes()
print(f"n={side * side} r={rank}: {out['done']} it in {out['seconds']:.3f}s; stages us {[round(x * 1e3, 1) for x in ms]} "
      f"GB/s {[round(b / (t * 1e-3) / 1e9) if t > 0 else 0 for b, t in zip(by, ms)]}; "
      f"auut {am * 1e3:.1f} us {ab / (am * 1e-3) / 1e9:.0f} GB/s", flush=True)
