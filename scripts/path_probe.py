#!/usr/bin/env python3
"""GPU box: fixed-rank ALM it/s of the BASELINE configs under each kernel path
(lrs_set_kernel_path 0 auto / 1 general row kernels / 2 + bandwidth-regime split / 3 + long-row
kernels) and the per-stage launch times, to check the planner's choice per instance."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
for name, rank in (("theta3", 26), ("theta3x3", 26), ("G1", 0), ("G22", 0)):
    pth = inst.config_instance(name, cache)
    for path in (0, 1, 2, 3):
        sv = solver.Solver(pth)
        sv.set_kernel_path(path)
        r = rank or sv.determine_rank()[0]
        kw = dict(fixedRank=r, reoptLevel=0)
        sv.alm_throughput(0, 200, **kw)
        o = sv.alm_throughput(0, 2000, **kw)
        ms = sv.time_stages(100)
        print(f"{name} r={r} path={path} ran={sv.kernel_path()}: {o['done'] / o['seconds']:.0f} it/s, stages us "
              f"{[round(x * 1e3, 2) for x in ms]}", flush=True)
        sv.close()
