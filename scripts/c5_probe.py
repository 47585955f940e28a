#!/usr/bin/env python3
"""Diagnostics (GPU box): BASELINE config C5 (random sparse SDP, n = 10^4, m = 10^6, k = 6
entries per constraint, r = 128) built in memory through lrs_load_coo; ALM it/s at fixed
rank, per-stage times / algorithmic GB/s, A(UU^T) and the MFMA Gram."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 128
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
t0 = time.time()
coo = inst.coo_arrays(inst.random_sparse_problem(n, m, 6, 5))
t1 = time.time()
sv = solver.Solver(coo=coo)
t2 = time.time()
print(f"gen {t1 - t0:.1f}s load {t2 - t1:.1f}s m={sv.m} slots={sv.nslots} nnz={sv.nnz}", flush=True)
out = sv.alm_throughput(2, iters, fixedRank=rank, reoptLevel=0)
print(f"alm {out['done']} it in {out['seconds']:.3f}s = {out['done'] / out['seconds']:.1f} it/s", flush=True)
ms = sv.time_stages(3)
by = sv.stage_bytes()
print(f"stages us {[round(x * 1e3, 1) for x in ms]} bytes {by} "
      f"GB/s {[round(b / (t * 1e-3) / 1e9) if t > 0 else 0 for b, t in zip(by, ms)]}", flush=True)
am = sv.time_auut(3)
ab = sv.auut_bytes()
print(f"auut {am * 1e3:.1f} us {ab / (am * 1e-3) / 1e9:.0f} GB/s", flush=True)
ms, kms = sv.time_gram(0, 20)
fl = sv.dims[0] * rank * (rank + 1)
print(f"gram r={rank}: {ms * 1e3:.1f} us incl. reduce, kernel {kms * 1e3:.1f} us = {fl / (kms * 1e-3) / 1e12:.2f} TFLOP/s",
      flush=True)
