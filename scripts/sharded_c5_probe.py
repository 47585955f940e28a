#!/usr/bin/env python3
"""Diagnostics (GPU box): BASELINE config C5 through the sharded iteration on a one-rank RCCL
communicator (run with LRS_FORCE_SHARD=1), a few timed ALM trips, for a kernel trace of what the
sharded path adds to the unsharded one."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 1000000, 6, 5)))
if len(sys.argv) < 2 or sys.argv[1] != "unsharded":
    sv.shard_rccl(1, 0, solver.comm_unique_id())
out = sv.alm_timed(3, 20, fixedRank=128, reoptLevel=0)
print(f"info {sv.shard_info()} tiles {sv.tile_used()} alm {out['done']} it in {out['seconds']:.4f}s = "
      f"{out['done'] / out['seconds']:.1f} it/s", flush=True)
sv.close()
