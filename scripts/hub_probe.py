#!/usr/bin/env python3
"""GPU box: one bundled instance solved on each kernel path (0 auto, 1 general), with the
library LRS_LIB names (default: the in-tree build).  One JSON line per solve.
Run:  [LRS_LIB=...] python scripts/hub_probe.py NAME [reoptLevel]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
name = sys.argv[1]
reopt = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for path in (0, 1):
    sv = solver.Solver(os.path.join(ROOT, "data", "bundled", f"{name}.dat-s"))
    sv.set_kernel_path(path)
    t0 = time.perf_counter()
    r = sv.solve(reoptLevel=reopt)
    t1 = time.perf_counter()
    kp = sv.kernel_path()
    sv.close()
    print(json.dumps({"lib": os.environ.get("LRS_LIB", "default"), "instance": name, "path": path, "taken": kp,
                      "sec": t1 - t0, **{k: r[k] for k in ("alm_inner", "admm_iter", "pobj", "dobj", "pinf", "gap",
                                                            "dinf", "status", "alm_pobj")}}), flush=True)
