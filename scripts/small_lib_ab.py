#!/usr/bin/env python3
"""GPU box A/B of two builds on the single-workgroup inner loop (k_small_alm): theta solves
(SDPLIB flags, bench.py's configs leg) with ltr-lowrank-sdp_amd/_build/liblrsdp_prev.so and with
the in-tree build, each solve in its own process (LRS_LIB), interleaved rounds.  Prints wall and
ALM-phase times and whether the two builds' trajectories are bit-identical (same inner count,
same primal objective bits)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build")
CHILD = r"""
import importlib, json, os, sys, time
sys.path.insert(0, {root!r})
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
cache = os.path.join({root!r}, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sv = solver.Solver(inst.config_instance({name!r}, cache))
t0 = time.perf_counter()
r = sv.solve(reoptLevel=0, heuristicFactor=1.0, phase1Tol=1e-3, rhoMax=5000.0)
wall = time.perf_counter() - t0
print(json.dumps(dict(wall=wall, alm=r["alm_time"], admm=r["admm_time"], inner=r["alm_inner"],
                      pobj=r["pobj"].hex())))
sv.close()
"""


def one(name, lib):
    env = dict(os.environ)
    if lib:
        env["LRS_LIB"] = lib
    else:
        env.pop("LRS_LIB", None)
    out = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, name=name)], env=env, capture_output=True,
                         text=True, timeout=180)
    if out.returncode != 0:
        raise SystemExit(out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


for name in sys.argv[1:] or ["theta3", "theta3x3"]:
    res = {"prev": [], "main": []}
    for rnd in range(3):
        for tag, lib in (("prev", os.path.join(BUILD, "liblrsdp_prev.so")), ("main", None)):
            r = one(name, lib)
            res[tag].append(r)
            print(name, tag, rnd, json.dumps(r), flush=True)
    same = all(a["inner"] == b["inner"] and a["pobj"] == b["pobj"] for a, b in zip(res["prev"], res["main"]))
    print(f"{name}: best wall prev {min(r['wall'] for r in res['prev']):.4f} s main "
          f"{min(r['wall'] for r in res['main']):.4f} s; best alm prev {min(r['alm'] for r in res['prev']):.4f} s "
          f"main {min(r['alm'] for r in res['main']):.4f} s; bit-identical trajectories: {same}", flush=True)
