#!/usr/bin/env python3
"""Diagnostics (GPU box): per-stage launch times of the split ALM iteration on a config
instance (ltr-lowrank-sdp_amd/instances.py CONFIGS).  usage: stage_probe.py NAME [RANK]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
for name in sys.argv[1:]:
    rank = 0
    if ":" in name:
        name, rank = name.split(":")
        rank = int(rank)
    sv = solver.Solver(inst.config_instance(name, cache))
    r = rank or sv.determine_rank()[0]
    sv.alm_throughput(0, 100, fixedRank=r, reoptLevel=0)
    out = sv.alm_throughput(0, 1000, fixedRank=r, reoptLevel=0)
    ms = sv.time_stages(100)
    by = sv.stage_bytes()
    am = sv.time_auut(100)
    print(f"{name} n={sv.dims} m={sv.m} slots={sv.nslots} r={r}: {out['done'] / out['seconds']:.0f} it/s; "
          f"stages A/G/B us {[round(x * 1e3, 1) for x in ms]}; GB/s "
          f"{[round(b / (t * 1e-3) / 1e9) if t > 0 else 0 for b, t in zip(by, ms)]}; auut {am * 1e3:.1f} us",
          flush=True)
    sv.close()
