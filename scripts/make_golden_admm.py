#!/usr/bin/env python3
"""Golden fixtures for the per-cone / per-side ADMM operator and the dual update at the C-ABI
(include/lrsdp.h lrs_op_admm_half(ctx, cone, side, ...), lrs_op_dual_update), from the
REFERENCE itself: oracle/_ref/lorads_ref_harness admm_sweep runs LORADSUpdateSDPVar
(lorads_alg_common.c:298-326: every cone, U with V fixed then V with U fixed, each followed by
the cone's constraint-value refresh) and LORADSUpdateDualVar (:511-524) on the inputs of the
kernels_<name>.npz fixtures (U, V, lambda, rho_admm, cg_tol).

Writes tests/golden/admm_sweep_<name>.npz: U, V after the sweep (column-major per cone, cones
concatenated), cvs (A(UV^T) summed over cones), lam (after the dual update), cg_total and the
last CG count of every cone.  Run:  python scripts/make_golden_admm.py  (needs /root/reference)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
NAMES = ["theta25x3", "mc_rand200", "rsparse60", "theta40"]
# the kernels fixtures' cg_tol (1e-12) sits at the rounding floor of ||r||_2 / ||b||_1, where CG
# iteration counts follow the rounding; the sweep is pinned at a tolerance the ADMM phase itself
# reaches (its CG tol is min(1e-2 pinf, 1e-8), lorads_admm.c:127)
CG_TOL = 1e-9


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference first: make -C oracle -f Makefile.ref")
    with tempfile.TemporaryDirectory() as td:
        for name in NAMES:
            k = np.load(os.path.join(GOLD, f"kernels_{name}.npz"))
            vec, rank, m, dims = k["inputs"].copy(), int(k["rank"]), int(k["m"]), [int(d) for d in k["dims"]]
            NR = sum(d * rank for d in dims)
            vec[9 * NR + 2 * m + 4] = CG_TOL
            fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
            vec.astype(np.float64).tofile(fin)
            path = os.path.join(GOLD, "instances", f"{name}.dat-s")
            subprocess.run([HARNESS, "admm_sweep", path, str(rank), fin, fout], check=True,
                           stdout=subprocess.DEVNULL, cwd=td)
            out = np.fromfile(fout, dtype=np.float64)
            p = 0
            U = out[p:p + NR]; p += NR
            V = out[p:p + NR]; p += NR
            cvs = out[p:p + m]; p += m
            lam = out[p:p + m]; p += m
            cg_total = out[p]; p += 1
            cg_last = out[p:p + len(dims)]; p += len(dims)
            assert p == out.size, (p, out.size)
            np.savez_compressed(os.path.join(GOLD, f"admm_sweep_{name}.npz"), U=U, V=V, cvs=cvs, lam=lam,
                                cg_total=cg_total, cg_last=cg_last, rank=rank, m=m, dims=np.array(dims),
                                cg_tol=CG_TOL)
            print("admm_sweep", name, "cones", len(dims), "cg", cg_total, cg_last)


if __name__ == "__main__":
    main()
