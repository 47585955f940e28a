#!/usr/bin/env python3
"""Diagnostics (GPU box): the MFMA Gram R^T R (k_gram + k_gram_fin) on a torus MaxCut factor,
n = rows * cols, for a list of fixed ranks; prints us per Gram and TFLOP/s (n r (r+1))."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
if os.environ.get("LRS_LIB"):
    solver.load_library(os.environ["LRS_LIB"])
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
side = int(sys.argv[1]) if len(sys.argv) > 1 else 100
ranks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "19,64,128,256").split(",")]
path = f"/tmp/gram_torus_{side}.dat-s"
inst.maxcut_torus(path, side, side, seed=1)
for r in ranks:
    sv = solver.Solver(path)
    sv.alm_throughput(1, 2, fixedRank=r, reoptLevel=0)
    ms, kms = sv.time_gram(0, 50)
    fl = sv.dims[0] * r * (r + 1)
    print(f"gram n={sv.dims[0]} r={r}: {ms * 1e3:.2f} us = {fl / (ms * 1e-3) / 1e12:.2f} TFLOP/s "
          f"({fl / (ms * 1e-3) / 1e12 / 78.6:.3f} of 78.6); MFMA kernel alone {kms * 1e3:.2f} us "
          f"({fl / (kms * 1e-3) / 1e12 / 78.6:.3f})", flush=True)
    sv.close()
sv = solver.Solver(path)
print(f"measured FP64 MFMA ceiling: {sv.mfma_f64_peak():.1f} TFLOP/s", flush=True)
sv.close()
