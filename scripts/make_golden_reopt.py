#!/usr/bin/env python3
"""Golden fixtures for reoptLevel 1 (main.c:491-513, reopt() data/lorads_solver.c:1497-1539)
from the REFERENCE itself: oracle/_ref/lorads_ref_harness (our driver over the reference
objects built by oracle/Makefile.ref) runs the committed instances with --reoptLevel 1 and
--reoptLevel 0; tests/golden/solves_reopt.json keeps the REF_RESULT values and the JSON
metrics of both.  Level 2 needs the ARPACK dual infeasibility, which the image lacks (no
fixture).  Run: python scripts/make_golden_reopt.py   (CPU only, needs /root/reference built)
"""
import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
CASES = ["theta40", "rsparse60", "theta25x3", "mc_rand200"]


def run(path, level, td):
    js = os.path.join(td, "o.json")
    r = subprocess.run([HARNESS, "solve", path, "--reoptLevel", str(level), "--jsonfile", js], capture_output=True,
                       text=True, cwd=td, check=True, env=dict(os.environ, OPENBLAS_NUM_THREADS="1"))
    res = {}
    for line in r.stdout.splitlines():
        if line.startswith("REF_RESULT"):
            for kv in line.split()[1:]:
                k, v = kv.split("=")
                res[k] = float(v)
    res["reopt_entered_admm"] = int("enter admm reopt" in r.stdout)
    with open(js) as f:
        metrics = json.load(f)["metrics"]
    return res, metrics


def main():
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name in CASES:
            path = os.path.join(GOLD, "instances", f"{name}.dat-s")
            r1, m1 = run(path, 1, td)
            r0, _ = run(path, 0, td)
            out.append({"instance": name, "flags": ["--reoptLevel", "1"], "result": r1, "metrics": m1,
                        "level0_alm_outer": r0["alm_outer"]})
            print(name, {k: r1[k] for k in ("alm_outer", "alm_pobj", "admm_iter", "admm_gap", "admm_pinf")},
                  "level-0 alm_outer", r0["alm_outer"])
    with open(os.path.join(GOLD, "solves_reopt.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
