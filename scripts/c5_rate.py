#!/usr/bin/env python3
"""GPU box: BASELINE config C5 (n = 1e4, m = 1e6, r = 128, in memory) ALM it/s as bench.py's
config_c5 times it (alm_timed: 3 warmup trips, then 20 timed ones of the same solve), with the
outer-iteration constraint evaluation on the constraint-entry tiles (default) and on the
pattern SDDMM + gather (LRS_CONSTR_TILES=0), each twice, one load."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
dense = len(sys.argv) > 1 and sys.argv[1] == "c5b"
sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5, dense_c=dense)))
for v in ("1", "0", "1", "0"):
    os.environ["LRS_CONSTR_TILES"] = v
    o = sv.alm_timed(3, 20, fixedRank=128, reoptLevel=0)
    print(f"{'c5b' if dense else 'c5'} LRS_CONSTR_TILES={v}: {o['done']} it in {o['seconds']:.4f} s = "
          f"{o['done'] / o['seconds']:.1f} it/s", flush=True)
sv.close()
