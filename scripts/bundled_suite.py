#!/usr/bin/env python3
"""GPU box: the reference's own bundled instances (data/bundled/) solved on the device, with
(a) the flags of the golden reference solves (tests/golden/solves_bundled.json) and (b) the
flags of the reference's published runs (lorads/scripts/run.ipynb: General SDP
"--reoptLevel 2 --timeSecLimit 10000"; Gset: README.md:166).  One JSON line per solve."""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
DATA = os.path.join(ROOT, "data", "bundled")
GSET = dict(reoptLevel=0, heuristicFactor=10.0, phase1Tol=1e-2)
GENERAL_PUBLISHED = dict(reoptLevel=2, timeSecLimit=10000.0)
CASES = [("G11", GSET, GSET), ("G12", GSET, GSET), ("G13", GSET, GSET),
         ("cphil12", dict(reoptLevel=0), GENERAL_PUBLISHED),
         ("checker_1.5", dict(reoptLevel=0), GENERAL_PUBLISHED),
         ("ice_2.0", dict(reoptLevel=0), GENERAL_PUBLISHED),
         ("p_auss2_3.0", dict(reoptLevel=0), GENERAL_PUBLISHED),
         ("theta102", dict(reoptLevel=0), GENERAL_PUBLISHED),
         ("MC_500", dict(reoptLevel=0), GENERAL_PUBLISHED)]
want = set(sys.argv[1:])
for name, gflags, pflags in CASES:
    if want and name not in want:
        continue
    for tag, kw in (("golden_flags", gflags), ("published_flags", pflags)):
        if tag == "published_flags" and pflags is gflags:
            continue
        t0 = time.perf_counter()
        sv = solver.Solver(os.path.join(DATA, f"{name}.dat-s"))
        t1 = time.perf_counter()
        r = sv.solve(**kw)
        t2 = time.perf_counter()
        sv.close()
        keep = ("alm_inner", "admm_iter", "pobj", "dobj", "pinf", "gap", "dinf", "dinf_inf", "status", "final_rank",
                "solve_time", "alm_pobj")
        print(json.dumps({"instance": name, "run": tag, "flags": kw, "load_sec": t1 - t0, "call_sec": t2 - t1,
                          **{k: r[k] for k in keep}}), flush=True)
