#!/usr/bin/env python3
"""GPU box: the C5b dense product C R (n = 1e4, r = 128) per launch and its FP64 MFMA rate."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, 100000, 6, 5, dense_c=True)))
sv.alm_steps(1, fixedRank=128, reoptLevel=0)
for _ in range(2):
    ms = sv.time_dense(0, 10)
    print("C R %.1f us, %.1f TFLOP/s (%.3f of 78.6)" % (ms * 1e3, 2.56e10 / (ms * 1e-3) / 1e12,
                                                      2.56e10 / (ms * 1e-3) / 1e12 / 78.6), flush=True)
sv.close()
