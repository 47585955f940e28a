#!/usr/bin/env python3
"""Golden fixtures of LoRADS's LP cone (an SDPA block of negative size: data/lorads_lp_conic.c,
data/lorads_lp_data.c, the *LP variants bound in data/lorads_solver.c:1014-1053), from the
REFERENCE itself (oracle/_ref/lorads_ref_harness, our driver over the reference objects):

* tests/golden/admm_sweep_lp_<name>.npz -- `admm_sweep_lp`: LORADSUpdateSDPLPVar
  (lorads_alg_common.c:352-372: the SDP cones' CG half-steps, then the LP columns' closed-form
  updates, lorads_admm.c:759-792) and LORADSUpdateDualVar on seeded U, V, lambda; U / V hold the
  LP block's values after the SDP cones' (the device's LP cone at rank 1).
* tests/golden/solves_lp.json -- whole solves (REF_RESULT, the ALM log and the --jsonfile output)
  of instances.maxcut_lp (tests/golden/instances/mc_lp60.dat-s) and of the reference's own bundled
  shmup4 (2 SDP blocks + an LP block of 1 600 columns; data/bundled/shmup4.dat-s), --reoptLevel 0
  (benchmark.py's setting).  shmup4 takes a few minutes on one core.
The per-trip fixture of mc_lp60 is scripts/make_golden_steps.py's.
Run:  python scripts/make_golden_lp.py [sweep|solves]  (needs /root/reference; CPU only)"""
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
LINE = re.compile(r"ALM OuterIter:(\d+) InnerIter:(\d+) pObj:(\S+) dObj:(\S+) pInfea\(1\):(\S+)")
SOLVES = [("mc_lp60", os.path.join(GOLD, "instances", "mc_lp60.dat-s"), ["--reoptLevel", "0"]),
          ("shmup4", os.path.join(ROOT, "data", "bundled", "shmup4.dat-s"), ["--reoptLevel", "0"])]
ENV = dict(os.environ, OPENBLAS_NUM_THREADS="1")


def sweep(name, rank, dims_sdp, nlp, m, seed=3, cg_tol=1e-9, rho=2.0):
    rng = np.random.default_rng(seed)
    NA = sum(n * rank for n in dims_sdp) + nlp
    U = rng.standard_normal(NA)
    V = U + 0.1 * rng.standard_normal(NA)
    lam = rng.standard_normal(m)
    vec = np.concatenate([U, V, lam, [rho, cg_tol]])
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        vec.tofile(fi)
        r = subprocess.run([HARNESS, "admm_sweep_lp", os.path.join(GOLD, "instances", f"{name}.dat-s"), str(rank), fi,
                            fo], capture_output=True, text=True, env=ENV, cwd=td)
        assert r.returncode == 0, r.stdout + r.stderr
        out = np.fromfile(fo)
    p = 0
    U1 = out[p:p + NA]; p += NA
    V1 = out[p:p + NA]; p += NA
    cvs = out[p:p + m]; p += m
    lam1 = out[p:p + m]; p += m
    cg = out[p]; p += 1
    assert p == out.size
    np.savez_compressed(os.path.join(GOLD, f"admm_sweep_lp_{name}.npz"), U0=U, V0=V, lam0=lam, rho=rho, cg_tol=cg_tol,
                        U=U1, V=V1, cvs=cvs, lam=lam1, cg_total=cg, rank=rank, m=m, dims=np.array(dims_sdp + [nlp]))
    print("admm_sweep_lp", name, "cg", cg)


def solves():
    out = []
    for name, path, flags in SOLVES:
        with tempfile.TemporaryDirectory() as td:
            js = os.path.join(td, "o.json")
            t0 = time.time()
            r = subprocess.run([HARNESS, "solve", path, *flags, "--jsonfile", js], capture_output=True, text=True,
                               cwd=td, env=ENV)
            wall = time.time() - t0
            res = {}
            for line in r.stdout.splitlines():
                if line.startswith("REF_RESULT"):
                    for kv in line.split()[1:]:
                        k, v = kv.split("=")
                        res[k] = float(v)
            log = [[int(a), int(b), float(c), float(d), float(e)] for a, b, c, d, e in LINE.findall(r.stdout)]
            out.append({"instance": name, "flags": flags, "result": res, "alm_log": log, "wall_sec": wall,
                        "json": json.load(open(js))})
            print(name, {k: res.get(k) for k in ("alm_inner", "admm_iter", "alm_pobj", "admm_pobj", "admm_gap")},
                  f"wall {wall:.1f}s", flush=True)
    json.dump(out, open(os.path.join(GOLD, "solves_lp.json"), "w"), indent=1)


if __name__ == "__main__":
    what = sys.argv[1:] or ["sweep", "solves"]
    if "sweep" in what:
        sweep("mc_lp60", 9, [60], 63, 61)
    if "solves" in what:
        solves()
