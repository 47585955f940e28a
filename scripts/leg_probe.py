#!/usr/bin/env python3
"""One bench leg alone, for rocprofv3 (scripts/leg_profile.sh): build the leg's instance the way
bench.py does, run a few ALM trips to reach a steady state, then -- after an idle gap the
summariser splits the kernel trace on -- time the split-iteration stages (lrs_time_stages,
`reps` back-to-back relaunches per stage, LRS_TIME_STAGES_GAP_US idle gaps between stages) and
A(UU^T) (lrs_time_auut, `reps` relaunches).  Prints one JSON line with the HIP-event times and the
algorithmic bytes, which the summary puts beside the rocprof per-kernel sums.

usage: leg_probe.py {g67|g81|c5|torus2000} [reps]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
bench = importlib.import_module("bench")

if os.environ.get("LRS_LIB"):   # A/B of a variant build (ltr-lowrank-sdp_amd/_build/liblrsdp_<v>.so)
    solver.load_library(os.environ["LRS_LIB"])
leg = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
if leg == "g67":
    sv = solver.Solver(bench.instance_for(0, 100, 100, cache))
    rank, warm = sv.determine_rank()[0], 300
elif leg == "g81":
    sv = solver.Solver(bench.instance_for(0, 100, 200, cache, seed0=81))
    rank, warm = 64, 100
elif leg == "c5":
    sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5)))
    rank, warm = 128, 3
elif leg == "torus2000":
    sv = solver.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(2000, 2000, 2000)))
    rank, warm = 16, 5
else:
    raise SystemExit(f"unknown leg {leg}")
o = sv.alm_timed(warm, 5, fixedRank=rank, reoptLevel=0)
sv.sync()
time.sleep(0.5)                     # the gap in front of the timed region
os.environ.setdefault("LRS_TIME_STAGES_GAP_US", "200000")
ms = sv.time_stages(reps)
sv.sync()
time.sleep(0.2)                     # stage B | A(UU^T)
am = sv.time_auut(reps)
sv.sync()
print(json.dumps({"leg": leg, "rank": rank, "reps": reps, "kernel_path": sv.kernel_path(),
                  "stage_us": [x * 1e3 for x in ms], "stage_bytes": list(sv.stage_bytes()),
                  "auut_us": am * 1e3, "auut_bytes": sv.auut_bytes(), "it_s": o["done"] / o["seconds"]}), flush=True)
sv.close()
