#!/usr/bin/env python3
"""GPU box: A/B of library builds on the headline G67 leg (the latency kernels): bench-style ALM
it/s over 3 000 trips at the fixed rank 19 and lrs_time_stages per stage, each library in its own
process (LRS_LIB), interleaved rounds.  argv: variant names (main = the product build)."""
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
td = tempfile.mkdtemp()
p = os.path.join(td, "g67.dat-s")
inst.maxcut_torus(p, 100, 100, seed=67)
sv = solver.Solver(p)
kw = dict(fixedRank=19, reoptLevel=0)
sv.alm_throughput(0, 300, **kw)
o = sv.alm_throughput(0, 3000, **kw)
ms = sv.time_stages(200)
print(f"{os.environ['TAG']} g67: {o['done'] / o['seconds']:.0f} it/s stages us {[round(x * 1e3, 2) for x in ms]} path {sv.kernel_path()}", flush=True)
sv.close()
'''
names = sys.argv[1:] or ["main"]
for rnd in range(3):
    for nm in names:
        env = dict(os.environ, ROOT=ROOT, TAG=f"r{rnd} {nm}")
        if nm != "main":
            env["LRS_LIB"] = os.path.join(BUILD, f"liblrsdp_{nm}.so")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        sys.stdout.write(r.stdout)
        if r.returncode != 0:
            sys.stdout.write(f"{nm} failed: {r.stderr[-800:]}\n")
        sys.stdout.flush()
