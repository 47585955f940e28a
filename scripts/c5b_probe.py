#!/usr/bin/env python3
"""Diagnostics (GPU box): BASELINE config C5b (C5 with C a dense random symmetric matrix,
N(0, 1/n) + n I) built in memory; ALM it/s at fixed rank on the dense-objective path, per-stage
times, and the C R product on the matrix cores (2 n^2 r flop)."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 128
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
t0 = time.time()
coo = inst.coo_arrays(inst.random_sparse_problem(n, m, 6, 5, dense_c=True))
t1 = time.time()
sv = solver.Solver(coo=coo)
del coo
t2 = time.time()
print(f"gen {t1 - t0:.1f}s load {t2 - t1:.1f}s m={sv.m} slots={sv.nslots} nnz={sv.nnz}", flush=True)
out = sv.alm_throughput(2, iters, fixedRank=rank, reoptLevel=0)
print(f"alm {out['done']} it in {out['seconds']:.3f}s = {out['done'] / out['seconds']:.1f} it/s", flush=True)
ms = sv.time_stages(3)
print(f"stages us {[round(x * 1e3, 1) for x in ms]}", flush=True)
if os.environ.get("LRS_DENSE_C") == "0":
    sys.exit(0)
dm = sv.time_dense(0, 10)
fl = 2.0 * n * n * rank
peak = sv.mfma_f64_peak()
print(f"C R: {dm * 1e3:.1f} us = {fl / (dm * 1e-3) / 1e12:.2f} TFLOP/s ({fl / (dm * 1e-3) / 1e12 / 78.6:.3f} of 78.6, "
      f"{fl / (dm * 1e-3) / 1e12 / peak:.3f} of the measured {peak:.1f})", flush=True)
