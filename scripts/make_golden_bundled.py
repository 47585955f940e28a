#!/usr/bin/env python3
"""Golden solves of the reference on the instances it ships itself (lorads/data/General_SDP,
lorads/data/Max_cut_SDP,
lorads/data/Matrix_Completion_SDP; copied as data into data/bundled/): the reference LoRADS C code built
by oracle/Makefile.ref (oracle/_ref/lorads_ref_harness) solves each with the flags below and
the REF_RESULT line + JSON go to tests/golden/solves_bundled.json; the general SDPs' final
iterates (R, lambda; REF_DUMP) to tests/golden/bundled_final_<name>.npz.  reoptLevel 0 / 1 only: the
reference built here has no ARPACK, so its level-2 rounds (driven by the dual infeasibility)
are not the reference's.  CPU only; needs /root/reference.
Run:  python scripts/make_golden_bundled.py [name ...]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
DATA = os.path.join(ROOT, "data", "bundled")
OUT = os.path.join(ROOT, "tests", "golden", "solves_bundled.json")
GSET = ["--reoptLevel", "0", "--heuristicFactor", "10", "--phase1Tol", "1e-2"]   # lorads/README.md:166
CASES = [("G11", GSET), ("G12", GSET), ("G13", GSET),
         ("cphil12", ["--reoptLevel", "0"]), ("checker_1.5", ["--reoptLevel", "0"]),
         ("ice_2.0", ["--reoptLevel", "0"]), ("p_auss2_3.0", ["--reoptLevel", "0"]),
         ("theta102", ["--reoptLevel", "0"]), ("MC_500", ["--reoptLevel", "0"])]


DUMP = ("checker_1.5", "ice_2.0", "p_auss2_3.0")   # general SDPs: their final iterates (tests/test_bundled.py)


def save_final(dump, out):
    """REF_DUMP layout (oracle/ref_harness.c): {K, ranks[K], R (cones concatenated), m, lambda[m]}."""
    import numpy as np
    v = np.fromfile(dump, dtype=np.float64)
    K = int(v[0])
    rest = v.size - 1 - K
    m = next(c for c in range(1, rest) if v[1 + K + rest - 1 - c] == c)
    NR = rest - 1 - m
    np.savez_compressed(out, ranks=v[1:1 + K].astype(np.int64), R=v[1 + K:1 + K + NR], lam=v[2 + K + NR:], m=m)


def main():
    want = set(sys.argv[1:])
    old = json.load(open(OUT)) if os.path.exists(OUT) else []
    keep = [o for o in old if want and o["instance"] not in want]
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    with tempfile.TemporaryDirectory() as td:
        for name, flags in CASES:
            if want and name not in want:
                continue
            path = os.path.join(DATA, f"{name}.dat-s")
            js = os.path.join(td, "o.json")
            dump = os.path.join(td, f"{name}.final")
            env_run = dict(env, REF_DUMP=dump) if name in DUMP else env
            t0 = time.time()
            r = subprocess.run([HARNESS, "solve", path, *flags, "--timeSecLimit", "1800", "--jsonfile", js],
                               capture_output=True, text=True, cwd=td, env=env_run)
            if os.path.exists(dump):   # the final iterate (R per cone, lambda) for the device's certificate check
                save_final(dump, os.path.join(ROOT, "tests", "golden", f"bundled_final_{name}.npz"))
            wall = time.time() - t0
            res = {}
            for line in r.stdout.splitlines():
                if line.startswith("REF_RESULT"):
                    for kv in line.split()[1:]:
                        k, v = kv.split("=")
                        res[k] = float(v)
            if not res:
                print("no result", name, r.stdout[-2000:], r.stderr[-2000:])
                continue
            ref_json = json.load(open(js)) if os.path.exists(js) else None
            keep.append({"instance": name, "flags": flags, "result": res, "wall_sec": wall, "json": ref_json})
            print(name, flags, {k: res.get(k) for k in ("alm_inner", "admm_pobj", "admm_dobj", "solve_time")},
                  f"wall {wall:.1f}s", flush=True)
            json.dump(keep, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
