#!/usr/bin/env python3
"""GPU box: the FP64 MFMA probe over occupancy (waves per SIMD) and independent chains, with the
shader clock under load and the cycles per v_mfma_f64_16x16x4f64 per SIMD."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
G = os.path.join(ROOT, "tests", "golden", "instances", "mc_rand200.dat-s")
sv = solver.Solver(G)
for wps in (1, 2, 4, 8):
    for ch in (4, 8):
        t, f, cy = sv.mfma_f64_probe(wps, ch)
        print(f"waves/SIMD {wps} chains {ch}: {t:.1f} TFLOP/s, {f:.0f} MHz under load, {cy:.1f} cycles/MFMA/SIMD "
              f"(64 at the 78.6 TF spec)", flush=True)
sv.close()
