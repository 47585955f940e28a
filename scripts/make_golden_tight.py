#!/usr/bin/env python3
"""Reference solves of the general SDPs and theta3 at tighter tolerances than the
reference's default phase2Tol 1e-5 (main.c:75), so that the device's objectives can be
pinned beyond what the default stopping rule fixes; the tightest run's final iterate (R per cone,
lambda) goes to tests/golden/tight_final_<name>.npz (REF_DUMP, oracle/ref_harness.c) (checker_1.5 /
ice_2.0 / p_auss2_3.0 agree only to ~1e-4 at 1e-5).

The reference LoRADS C code built by oracle/Makefile.ref (oracle/_ref/lorads_ref_harness)
solves each instance with its usual flags plus --phase2Tol T for T in 1e-7, 1e-8; the
REF_RESULT line, the per-outer-iteration ALM log and the JSON go to
tests/golden/solves_tight.json.  CPU only; needs /root/reference (for the harness build).
Run:  python scripts/make_golden_tight.py [name ...]"""
import hashlib
import importlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
DATA = os.path.join(ROOT, "data", "bundled")
OUT = os.path.join(ROOT, "tests", "golden", "solves_tight.json")
SDPLIB = ["--reoptLevel", "0", "--heuristicFactor", "1.0", "--phase1Tol", "1e-3", "--rhoMax", "5000.0"]
CASES = [("checker_1.5", "bundled", ["--reoptLevel", "0"]),
         ("ice_2.0", "bundled", ["--reoptLevel", "0"]),
         ("p_auss2_3.0", "bundled", ["--reoptLevel", "0"]),
         ("theta3", "config", SDPLIB)]
TOLS = ["1e-7", "1e-8"]
LINE = re.compile(r"ALM OuterIter:(\d+) InnerIter:(\d+) pObj:(\S+) dObj:(\S+) pInfea\(1\):(\S+)")


def run_one(name, kind, flags, tol, td):
    if kind == "bundled":
        path = os.path.join(DATA, f"{name}.dat-s")
    else:
        inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
        d = os.path.join(td, f"{name}_{tol}")
        os.makedirs(d, exist_ok=True)
        path = inst.config_instance(name, d)
    sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
    js = os.path.join(td, f"{name}_{tol}.json")
    fl = [*flags, "--phase2Tol", tol]
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    dump = os.path.join(td, f"{name}_{tol}.final")
    if tol == TOLS[-1]:   # the tightest run's final iterate (R per cone, lambda) for the device check
        env["REF_DUMP"] = dump
    t0 = time.time()
    r = subprocess.run([HARNESS, "solve", path, *fl, "--timeSecLimit", "3000", "--jsonfile", js],
                       capture_output=True, text=True, cwd=td, env=env)
    wall = time.time() - t0
    res = {}
    for line in r.stdout.splitlines():
        if line.startswith("REF_RESULT"):
            for kv in line.split()[1:]:
                k, v = kv.split("=")
                res[k] = float(v)
    log = [[int(a), int(b), float(c), float(d), float(e)] for a, b, c, d, e in LINE.findall(r.stdout)]
    if os.path.exists(dump):
        # {K, ranks[K], R (cones concatenated), m, lambda[m]}: m is the count of the trailing block
        v = np.fromfile(dump, dtype=np.float64)
        K = int(v[0])
        ranks = v[1:1 + K].astype(np.int64)
        rest = v.size - 1 - K
        mm = next(c for c in range(1, rest) if v[1 + K + rest - 1 - c] == c)
        NR = rest - 1 - mm
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", f"tight_final_{name}.npz"), ranks=ranks,
                            R=v[1 + K:1 + K + NR], lam=v[2 + K + NR:], m=mm, tol=float(tol))
    out = {"instance": name, "kind": kind, "sha256": sha, "flags": fl, "result": res, "alm_log": log,
           "wall_sec": wall, "json": json.load(open(js)) if os.path.exists(js) else None}
    print(name, tol, {k: res.get(k) for k in ("alm_inner", "admm_iter", "admm_pobj", "admm_dobj", "admm_gap",
                                             "admm_pinf")}, f"wall {wall:.1f}s", flush=True)
    return out


def main():
    want = set(sys.argv[1:])
    old = json.load(open(OUT)) if os.path.exists(OUT) else []
    jobs = [(n, k, f, t) for n, k, f in CASES for t in TOLS if not want or n in want]
    keep = [o for o in old if (o["instance"], o["flags"][-1]) not in {(n, t) for n, _, _, t in jobs}]
    with tempfile.TemporaryDirectory() as td, ThreadPoolExecutor(4) as ex:
        futs = [ex.submit(run_one, n, k, f, t, td) for n, k, f, t in jobs]
        for fu in futs:
            keep.append(fu.result())
            keep.sort(key=lambda o: (o["instance"], o["flags"][-1]))
            json.dump(keep, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
