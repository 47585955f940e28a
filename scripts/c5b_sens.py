#!/usr/bin/env python3
"""GPU box: rounding sensitivity of the C5b trips (n = 1e4, m = 1e6, r = 128, dense C).  Runs
K = 1..3 trips with the split-K slab count of k_cgemm2 taken from LRS_CG_SPLIT (read once per
process: another C R summation order per value), prints the relative errors of the projected
R / G / s / y / cvs / lam against tests/golden/steps_c5b_m1e6.npz (the reference's own trips) and
saves the projections to argv[1] so that two processes' runs can be compared with each other."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_util import rel_err  # noqa: E402
from test_gpu_c5_steps import project_factor, project_mvec  # noqa: E402

solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
N = 10000
z = np.load(os.path.join(ROOT, "tests", "golden", "steps_c5b_m1e6.npz"))
sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(N, int(z["m"]), 6, 5, dense_c=True)))
out = {}
for K in (1, 2, 3):
    d = sv.alm_steps(K, reoptLevel=0, fixedRank=int(z["rank_flag"]))
    tau = z[f"K{K}_trips"][K - 1][0]
    errs = {"tau": abs(d["tau"] - tau) / abs(tau)}
    for key in ("R", "G", "s", "y", "cvs", "lam"):
        ours = project_mvec(d[key]) if key in ("cvs", "lam") else project_factor(d[key], N)
        out[f"K{K}_{key}"] = ours
        ref = z[f"K{K}_{key}"]
        errs[key] = rel_err(ours, ref) if np.linalg.norm(ref) > 0 else float(np.linalg.norm(ours))
    out[f"K{K}_tau"] = np.array([d["tau"]])
    print(f"LRS_CG_SPLIT={os.environ.get('LRS_CG_SPLIT', 'auto')} K={K} vs reference:",
          " ".join(f"{k} {v:.2e}" for k, v in errs.items()), flush=True)
sv.close()
np.savez(sys.argv[1], **out)
if len(sys.argv) > 2 and os.path.exists(sys.argv[2]):
    o = np.load(sys.argv[2])
    for K in (1, 2, 3):
        print(f"K={K} vs {os.path.basename(sys.argv[2])}:",
              " ".join(f"{k} {rel_err(out[f'K{K}_{k}'], o[f'K{K}_{k}']):.2e}" for k in ("tau", "R", "G", "s", "y", "cvs", "lam")))
