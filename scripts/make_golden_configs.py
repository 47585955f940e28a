#!/usr/bin/env python3
"""Golden solves of the reference for the remaining BASELINE.json configs: G1 (n = 800),
G22 (n = 2000, default rank 16), theta3 (n = 150, m = 1106) and a 3-block stack of theta3
(multi-cone), each with benchmark.py's flags for its subtype (get_lorads_params,
benchmark.py:136-200: Gset -> phase1Tol 1e-2, heuristicFactor 10; SDPLIB -> phase1Tol 1e-3,
heuristicFactor 1; both rhoMax 5000, reoptLevel 0) -- the same flags bench.py's
configs_wall_clock_to_eps uses.

The instances are ours (ltr-lowrank-sdp_amd/instances.py CONFIGS, written by
config_instance); only their sha256 is stored.  The reference LoRADS C code built by
oracle/Makefile.ref (oracle/_ref/lorads_ref_harness) solves each; its REF_RESULT line,
JSON (lorads_logging.c:618-712) and per-outer-iteration ALM log go to
tests/golden/solves_configs.json.  CPU only; needs /root/reference.
Run:  python scripts/make_golden_configs.py"""
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
OUT = os.path.join(ROOT, "tests", "golden", "solves_configs.json")
GSET = ["--reoptLevel", "0", "--heuristicFactor", "10.0", "--phase1Tol", "1e-2", "--rhoMax", "5000.0"]
SDPLIB = ["--reoptLevel", "0", "--heuristicFactor", "1.0", "--phase1Tol", "1e-3", "--rhoMax", "5000.0"]
CASES = [("G1", GSET), ("G22", GSET), ("theta3", SDPLIB), ("theta3x3", SDPLIB)]
LINE = re.compile(r"ALM OuterIter:(\d+) InnerIter:(\d+) pObj:(\S+) dObj:(\S+) pInfea\(1\):(\S+)")


def main():
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, flags in CASES:
            path = inst.config_instance(name, td)
            sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
            js = os.path.join(td, "o.json")
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
            out.append({"config": name, "spec": inst.CONFIGS[name], "sha256": sha, "flags": flags,
                        "result": res, "alm_log": log, "wall_sec": wall, "json": json.load(open(js))})
            print(name, {k: res.get(k) for k in ("alm_inner", "admm_iter", "alm_pobj", "admm_pobj", "admm_gap",
                                                 "solve_time")}, f"wall {wall:.1f}s", flush=True)
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
