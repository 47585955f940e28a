#!/usr/bin/env python3
"""Golden solves of the reference at the BASELINE.json headline sizes: the G67-structured
torus 100x100 (n = m = 10 000, the bench workload, default rank 19) and the G81-structured
torus 100x200 (n = m = 20 000) at the north-star's --fixedRank 64 and at the default rank.

The instances are ours (ltr-lowrank-sdp_amd/instances.py `maxcut_torus`, the seeds bench.py
uses); only their sha256 is stored so the test can check it regenerated the same file.  The
reference LoRADS C code built by oracle/Makefile.ref (oracle/_ref/lorads_ref_harness) solves
each with the Gset flags of lorads/README.md:166 (benchmark.py:136-200's Gset subtype) and the
REF_RESULT line, its JSON (lorads_logging.c:618-712) and its per-outer-iteration ALM log go to
tests/golden/solves_northstar.json.  CPU only; needs /root/reference.
Run:  python scripts/make_golden_northstar.py"""
import hashlib
import importlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
OUT = os.path.join(ROOT, "tests", "golden", "solves_northstar.json")
GSET = ["--reoptLevel", "0", "--heuristicFactor", "10", "--phase1Tol", "1e-2"]
# (name, rows, cols, seed, extra flags)
CASES = [("g67_torus100x100", 100, 100, 67, []),
         ("g81_torus100x200_r64", 100, 200, 81, ["--fixedRank", "64"]),
         ("g81_torus100x200", 100, 200, 81, [])]
LINE = re.compile(r"ALM OuterIter:(\d+) InnerIter:(\d+) pObj:(\S+) dObj:(\S+) pInfea\(1\):(\S+)")


def main():
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, rows, cols, seed, extra in CASES:
            path = os.path.join(td, f"{name}.dat-s")
            inst.maxcut_torus(path, rows, cols, seed=seed)
            sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
            js = os.path.join(td, "o.json")
            flags = GSET + extra
            t0 = time.time()
            r = subprocess.run([HARNESS, "solve", path, *flags, "--jsonfile", js], capture_output=True, text=True,
                               cwd=td, env=env)
            wall = time.time() - t0
            res = {}
            for line in r.stdout.splitlines():
                if line.startswith("REF_RESULT"):
                    for kv in line.split()[1:]:
                        k, v = kv.split("=")
                        res[k] = float(v)
            log = [[int(a), int(b), float(c), float(d), float(e)] for a, b, c, d, e in LINE.findall(r.stdout)]
            out.append({"instance": name, "rows": rows, "cols": cols, "seed": seed, "sha256": sha, "flags": flags,
                        "result": res, "alm_log": log, "wall_sec": wall, "json": json.load(open(js))})
            print(name, {k: res.get(k) for k in ("alm_inner", "alm_pobj", "admm_pobj", "solve_time")},
                  f"wall {wall:.1f}s", flush=True)
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
