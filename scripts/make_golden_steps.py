#!/usr/bin/env python3
"""Per-iteration golden fixtures of the ALM inner loop, from the REFERENCE itself.

Runs `oracle/_ref/lorads_ref_harness alm_steps` (our driver over the reference
LoRADS objects built by oracle/Makefile.ref): from the reference's own initial
point (srand(925), data/lorads_solver.c:625) the preamble of LORADS_ALMOptimize
(lorads_alm.c:1233-1243) and exactly K trips of the inner L-BFGS loop
(lorads_alm.c:1302-1379).  For every K in KS it stores

  trips[K, 4]  per trip: tau, rootNum, ||G||^2 after the trip, pinf after the trip
  R, G         the factor and gradient after trip K (col-major per cone, cones concatenated)
  cvs, lam     A(RR^T) and lambda after trip K
  s, y, beta   the newest L-BFGS pair (s = tau D, y = G_new - G_old, 1/<y,s>)

into tests/golden/steps_<name>.npz (data only; the instances are ours).
Run:  python scripts/make_golden_steps.py   (needs /root/reference; CPU only)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")

# (name, instance path, rank (-1 = the reference's default), Ks)
CASES = [
    ("mc_rand200", os.path.join(GOLD, "instances", "mc_rand200.dat-s"), -1, [1, 2, 3, 4, 5]),
    ("mc_torus12x10", os.path.join(GOLD, "instances", "mc_torus12x10.dat-s"), -1, [1, 2, 3, 4, 5]),
    ("mc_rand300w", os.path.join(GOLD, "instances", "mc_rand300w.dat-s"), 12, [1, 2, 3, 4, 5]),
    ("theta40", os.path.join(GOLD, "instances", "theta40.dat-s"), -1, [1, 2, 3, 4, 5]),
    ("theta25x3", os.path.join(GOLD, "instances", "theta25x3.dat-s"), -1, [1, 2, 3, 4, 5]),
    ("rsparse60", os.path.join(GOLD, "instances", "rsparse60.dat-s"), -1, [1, 2, 3, 4, 5]),
    # the reference's own bundled instance with hub rows (the latency kernels' slice blocks)
    ("checker_1.5", os.path.join(ROOT, "data", "bundled", "checker_1.5.dat-s"), -1, [1, 3, 5]),
    # rank 290 > 256 (the 64 x 8 layout): the n x r arrays stored as n x 4 projections R @ Omega
    ("mc_rand300w_r290", os.path.join(GOLD, "instances", "mc_rand300w.dat-s"), 290, [1, 2, 3, 5, 8]),
    # dense objective (C5b structure at test size, the reference's dense branches): the instance is
    # regenerated from ltr-lowrank-sdp_amd/instances.py random_sparse(300, 3000, 6, 7, dense_c=True)
    ("rdense300", "gen:rdense300", -1, [1, 2, 3, 4, 5]),
    # --lbfgsListLength other than 2 (data/lorads_solver.c:686-706, lorads_alm.c:468-505): a ring of 3
    # (a ring of 1 crashes the reference: its node links are only set in the loop that adds nodes 2..L)
    ("mc_rand200_l3", os.path.join(GOLD, "instances", "mc_rand200.dat-s"), -1, [1, 2, 3, 4, 5, 8]),
    ("theta40_l3", os.path.join(GOLD, "instances", "theta40.dat-s"), -1, [1, 2, 3, 4, 5, 8]),
    # an LP block (instances.maxcut_lp: slacks, a free variable split in two, a dense LP column): r and
    # its gradient appended after the SDP cone (the device's LP cone at rank 1), the pairs LP part last
    ("mc_lp60", os.path.join(GOLD, "instances", "mc_lp60.dat-s"), -1, [1, 2, 3, 4, 5, 8]),
]
FLAGS = {"mc_rand200_l3": ["--lbfgsListLength", "3"], "theta40_l3": ["--lbfgsListLength", "3"]}
GEN = {"rdense300": (300, 3000, 6, 7)}
PROJ = {"mc_rand300w_r290": 4}


def project(v, n, k, seed=7):
    """Col-major n x r array (one cone) -> (n x k) = V @ Omega, Omega ~ N(0,1) (r x k), seeded."""
    r = v.size // n
    om = np.random.default_rng(seed).standard_normal((r, k))
    return v.reshape(r, n).T @ om


def run_steps(path, rank, K, m, nr, flags=()):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "s.bin")
        r = subprocess.run([HARNESS, "alm_steps", path, str(rank), str(K), out, *flags], capture_output=True, text=True,
                           env=dict(os.environ, OPENBLAS_NUM_THREADS="1"), timeout=600)
        if r.returncode != 0 or "REF_STEPS" not in r.stdout:
            raise RuntimeError(r.stdout[-2000:] + r.stderr[-2000:])
        a = np.fromfile(out)
    done = int(a[0])
    p = 1
    trips = a[p:p + 4 * done].reshape(done, 4); p += 4 * done
    d = {"trips": trips}
    for key, ln in (("R", nr), ("G", nr), ("cvs", m), ("lam", m), ("s", nr), ("y", nr), ("beta", 1)):
        d[key] = a[p:p + ln]; p += ln
    assert p == a.size, (p, a.size)
    return d


def dims_of(path):
    """(m, block sizes) from the SDPA header."""
    with open(path) as f:
        lines = [ln for ln in f if ln.strip() and ln.lstrip()[0] not in '*"']
    m = int(lines[0].split()[0])
    nb = int(lines[1].split()[0])
    dims = [abs(int(x)) for x in lines[2].replace(",", " ").replace("{", " ").replace("}", " ")
            .replace("(", " ").replace(")", " ").split()[:nb]]
    return m, dims


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle -f Makefile.ref")
    only = set(sys.argv[1:])
    gen_dir = tempfile.TemporaryDirectory()
    for name, path, rank, ks in CASES:
        if only and name not in only:
            continue
        if path.startswith("gen:"):
            sys.path.insert(0, ROOT)
            import importlib
            inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
            path = os.path.join(gen_dir.name, f"{name}.dat-s")
            n_, m_, k_, seed_ = GEN[name]
            inst.random_sparse(path, n_, m_, k_, seed_, dense_c=True)
        m, dims = dims_of(path)
        # the reference's rank per cone is only known after presolve: read it back from R's size
        probe = None
        out = {}
        for K in ks:
            if probe is None:
                # first call with a generous nr guess; the dump's tail fixes the real size
                with tempfile.TemporaryDirectory() as td:
                    o = os.path.join(td, "s.bin")
                    subprocess.run([HARNESS, "alm_steps", path, str(rank), "1", o, *FLAGS.get(name, [])],
                                   capture_output=True, check=True,
                                   env=dict(os.environ, OPENBLAS_NUM_THREADS="1"), timeout=600)
                    a = np.fromfile(o)
                done = int(a[0])
                rest = a.size - 1 - 4 * done - 2 * m - 1
                assert rest % 4 == 0
                probe = rest // 4
            d = run_steps(path, rank, K, m, probe, FLAGS.get(name, []))
            for k, v in d.items():
                if name in PROJ and k in ("R", "G", "s", "y"):
                    v = project(v, dims[0], PROJ[name])
                out[f"K{K}_{k}"] = v
        out["ks"] = np.array(ks)
        out["m"] = np.array(m)
        out["dims"] = np.array(dims)
        out["nr"] = np.array(probe)
        out["rank_flag"] = np.array(rank)
        out["lbfgs_len"] = np.array(int(FLAGS.get(name, ["", "2"])[1]))
        np.savez_compressed(os.path.join(GOLD, f"steps_{name}.npz"), **out)
        t = out[f"K{ks[-1]}_trips"]
        print(f"{name}: m={m} dims={dims} nr={probe} taus={np.round(t[:, 0], 6).tolist()}")


if __name__ == "__main__":
    main()
