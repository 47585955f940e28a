#!/usr/bin/env python3
"""GPU box: the north-star workload (MaxCut torus 100 x 200 = G81 structure, n = m = 20 000,
--fixedRank 64): ALM it/s at fixed rank, per-stage launch times (lrs_time_stages) with their
algorithmic GB/s, and A(UU^T).  Environment switches (LRS_FOLD_MIN, ...) are read by the library."""
import importlib
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
td = tempfile.mkdtemp()
path = os.path.join(td, "g81.dat-s")
inst.maxcut_torus(path, 100, 200, seed=81)
sv = solver.Solver(path)
kw = dict(fixedRank=64, reoptLevel=0)
sv.alm_throughput(0, 100, **kw)
o = sv.alm_throughput(0, int(sys.argv[1]) if len(sys.argv) > 1 else 2000, **kw)
ms = sv.time_stages(100)
by = sv.stage_bytes()
am = sv.time_auut(200)
ab = sv.auut_bytes()
print(f"{os.environ.get('TAGV', '')} G81 r=64 path={sv.kernel_path()}: {o['done'] / o['seconds']:.0f} it/s; stages us "
      f"{[round(x * 1e3, 2) for x in ms]} GB/s {[round(b / (t * 1e-3) / 1e9) if t > 0 else 0 for b, t in zip(by, ms)]}; "
      f"auut {am * 1e3:.2f} us {ab / (am * 1e-3) / 1e9:.0f} GB/s", flush=True)
sv.close()
