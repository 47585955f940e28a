#!/usr/bin/env python3
"""GPU box: A/B of compile-time variants of the bandwidth-regime row kernels (LRS_BW_U: neighbours
in flight in stage A's second half k_it_a MODE 2; LRS_BW_UB: in the fused stage B k_it_b MODE 0)
on the G81-structured torus (r = 64) and the 2000^2 torus (r = 16): ALM it/s and per-stage times,
interleaved rounds, each library in its own process (LRS_LIB).  argv: variant names (main = the
product build)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build")
CHILD = r'''
import importlib, os, sys, tempfile
sys.path.insert(0, os.environ["ROOT"])
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
tag = os.environ["TAG"]
td = tempfile.mkdtemp()
p = os.path.join(td, "g81.dat-s")
inst.maxcut_torus(p, 100, 200, seed=81)
sv = solver.Solver(p)
kw = dict(fixedRank=64, reoptLevel=0)
sv.alm_throughput(0, 100, **kw)
o = sv.alm_throughput(0, 2000, **kw)
ms = sv.time_stages(100)
print(f"{tag} g81: {o['done'] / o['seconds']:.0f} it/s stages us {[round(x * 1e3, 2) for x in ms]}", flush=True)
sv.close()
if os.environ.get("BIG") == "1":
    sv = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(2000, 2000, 2000)))
    o = sv.alm_timed(5, 40, fixedRank=16, reoptLevel=0)
    ms = sv.time_stages(10)
    print(f"{tag} torus2000: {o['done'] / o['seconds']:.1f} it/s stages us {[round(x * 1e3, 1) for x in ms]}", flush=True)
    sv.close()
'''
names = sys.argv[1:] or ["main"]
for rnd in range(2):
    for nm in names:
        env = dict(os.environ, ROOT=ROOT, TAG=f"r{rnd} {nm}", BIG="1" if rnd == 0 else "0")
        if nm != "main":
            env["LRS_LIB"] = os.path.join(BUILD, f"liblrsdp_{nm}.so")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        sys.stdout.write(r.stdout)
        if r.returncode != 0:
            sys.stdout.write(f"{nm} failed: {r.stderr[-800:]}\n")
        sys.stdout.flush()
