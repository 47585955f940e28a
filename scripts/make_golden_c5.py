#!/usr/bin/env python3
"""Per-trip golden fixtures of the ALM inner loop on BASELINE config C5 (random sparse SDP,
n = 10^4, 6 entries per constraint, C = I, --fixedRank 128), from the REFERENCE itself.

`oracle/_ref/lorads_ref_harness alm_steps <file> 128 1,2,3 <out>` (our driver over the
reference LoRADS objects, oracle/Makefile.ref) runs the reference's initial point
(srand(925), data/lorads_solver.c:625), the preamble of LORADS_ALMOptimize
(lorads_alm.c:1233-1243) and K trips of its inner L-BFGS loop (lorads_alm.c:1302-1379),
dumping the state at every K of the list in ONE run (the reference's hash-chain presolve
at m = 10^6 takes ~25 minutes on one core).

Cases
  c5_m1e6   the full C5 instance (m = 10^6: pattern ~11.5 % of the lower triangle, so the
            reference takes its dense syr2k / symm branches; the device its 2-D LDS tiles)
  c5_m1e5   the same structure with m = 10^5 (reference sparse branches; the device's
            gather kernels by default, the tiles when forced)
  c5b_m1e6  C5b: the full C5 instance with C a dense random symmetric matrix (N(0, 1/n) + n I,
            the bench's config_c5b workload): the reference's dense dsyr2k / dsymm branches
            (lorads_alg_common.c:72-89, data/lorads_sdp_data.c:948-973) against the device's
            dense objective on the FP64 matrix cores (k_cgemm2) -- run with the reference's
            BLAS on 8 threads (OPENBLAS_NUM_THREADS, its n^2 r products)

The instance is regenerated from ltr-lowrank-sdp_amd/instances.py
random_sparse(10000, m, 6, 5) (the bench's config_c5 workload at m = 10^6) and its sha256
is stored.  n x r arrays (R, G, s, y; n = 10^4, r = 128) are stored as n x 2 projections
V @ Omega and m-vectors (A(RR^T), lambda) as every 997th entry plus 4 Gaussian projections
(fixture size; tests/test_gpu_c5_steps.py projects the device's arrays the same way).
Run:  python scripts/make_golden_c5.py [c5_m1e5] [c5_m1e6]   (CPU only, needs /root/reference)
"""
from __future__ import annotations

import hashlib
import importlib
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
N, K_ENT, SEED, RANK = 10000, 6, 5, 128
CASES = {"c5_m1e6": (1000000, [1, 2, 3]), "c5_m1e5": (100000, [1, 2, 3, 4, 5]),
         "c5b_m1e6": (1000000, [1, 2, 3])}
DENSE_C = {"c5b_m1e6"}
BLAS_THREADS = {"c5b_m1e6": "8"}
NPROJ_F, NPROJ_M, STRIDE_M = 2, 4, 997


def project_factor(v, n, k=NPROJ_F, seed=7):
    """Col-major n x r array -> n x k = V @ Omega, Omega ~ N(0,1) (r x k), seeded."""
    r = v.size // n
    om = np.random.default_rng(seed).standard_normal((r, k))
    return v.reshape(r, n).T @ om


def project_mvec(v, k=NPROJ_M, stride=STRIDE_M, seed=11):
    """m-vector -> every stride-th entry followed by k Gaussian projections."""
    om = np.random.default_rng(seed).standard_normal((k, v.size))
    return np.concatenate([v[::stride], om @ v])


def main():
    names = sys.argv[1:] or list(CASES)
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    for name in names:
        m, ks = CASES[name]
        env = dict(os.environ, OPENBLAS_NUM_THREADS=BLAS_THREADS.get(name, "1"))
        with tempfile.TemporaryDirectory(dir="/tmp") as td:
            path = os.path.join(td, f"{name}.dat-s")
            inst.random_sparse(path, N, m, K_ENT, SEED, dense_c=name in DENSE_C)
            sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
            out = os.path.join(td, "s.bin")
            t0 = time.time()
            r = subprocess.run([HARNESS, "alm_steps", path, str(RANK), ",".join(map(str, ks)), out],
                               capture_output=True, text=True, env=env)
            wall = time.time() - t0
            if r.returncode != 0:
                raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
            nr = N * RANK
            z = {"ks": np.array(ks), "m": np.array(m), "dims": np.array([N]), "rank_flag": np.array(RANK),
                 "sha256": np.array(sha), "wall_sec": np.array(wall), "dense_c": np.array(name in DENSE_C),
                 "blas_threads": np.array(int(env["OPENBLAS_NUM_THREADS"]))}
            for K in ks:
                a = np.fromfile(f"{out}.K{K}")
                done = int(a[0])
                p = 1
                z[f"K{K}_trips"] = a[p:p + 4 * done].reshape(done, 4)
                p += 4 * done
                for key, ln in (("R", nr), ("G", nr), ("cvs", m), ("lam", m), ("s", nr), ("y", nr), ("beta", 1)):
                    v = a[p:p + ln]
                    p += ln
                    if key in ("R", "G", "s", "y"):
                        v = project_factor(v, N)
                    elif key in ("cvs", "lam"):
                        v = project_mvec(v)
                    z[f"K{K}_{key}"] = v
                assert p == a.size, (p, a.size)
        np.savez_compressed(os.path.join(GOLD, f"steps_{name}.npz"), **z)
        t = z[f"K{ks[-1]}_trips"]
        print(f"{name}: m={m} wall {wall:.0f}s taus={t[:, 0].tolist()}", flush=True)


if __name__ == "__main__":
    main()
