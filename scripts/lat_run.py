#!/usr/bin/env python3
"""Diagnostics: the bench's headline ALM run (G67-like torus, default rank, phase-1 exit
off) for a rocprofv3 kernel trace; LRS_NO_LAT=1 selects the general row kernels."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
path = bench.instance_for(0, 100, 100, cache)
sv = solver.Solver(path)
r = sv.determine_rank()[0]
kw = dict(fixedRank=r, reoptLevel=0)
sv.alm_throughput(0, 300, **kw)
out = sv.alm_throughput(0, int(sys.argv[1]) if len(sys.argv) > 1 else 2000, **kw)
print(f"path={sv.kernel_path()} {out['done'] / out['seconds']:.1f} it/s")
sv.close()
