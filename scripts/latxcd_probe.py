#!/usr/bin/env python3
"""Diagnostics (GPU box): the G67 headline (latency kernels) with a library build given as
argv[1]: ALM it/s of one solve (alm_timed) -- run under rocprofv3 --pmc for its HBM bytes."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
solver.load_library(sys.argv[1])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
sv = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(100, 100, 67)))
r = sv.determine_rank()[0]
o = sv.alm_timed(300, steps, fixedRank=r, reoptLevel=0)
print(f"{os.path.basename(sys.argv[1])}: rank {r} {o['done'] / o['seconds']:.0f} it/s path {sv.kernel_path()}",
      flush=True)
sv.close()
