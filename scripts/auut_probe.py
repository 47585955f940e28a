#!/usr/bin/env python3
"""GPU box: A(U U^T) on the north-star G81-like torus (n = m = 20 000, r = 64): the event-timed
back-to-back launch average (bench.py's a_uut) -- run under rocprofv3 --kernel-trace --stats
for the kernel's own duration."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sv = solver.Solver(inst.config_instance("G81", cache))
sv.alm_throughput(0, 20, fixedRank=64, reoptLevel=0)
for reps in (200, 200):
    ms = sv.time_auut(reps)
    by = sv.auut_bytes()
    print("auut %.3f us per launch, %.1f MB, %.3f of 8 TB/s" % (ms * 1e3, by / 1e6, by / (ms * 1e-3) / 8e12), flush=True)
sv.close()
