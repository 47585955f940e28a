#!/usr/bin/env python3
"""Golden solves of the reference above rank 256 (the device's 64 x 8 factor layout, ld = 512):
the reference LoRADS C code built by oracle/Makefile.ref (oracle/_ref/lorads_ref_harness)
solves the committed instances with the flags below; REF_RESULT, the JSON and the ALM log
lines go to tests/golden/solves_highrank.json.  CPU only; needs /root/reference.
Run:  python scripts/make_golden_highrank.py"""
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "lorads_ref_harness")
INST = os.path.join(ROOT, "tests", "golden", "instances")
OUT = os.path.join(ROOT, "tests", "golden", "solves_highrank.json")
CASES = [("mc_rand300w", ["--reoptLevel", "0", "--fixedRank", "290"])]
LINE = re.compile(r"ALM OuterIter:(\d+) InnerIter:(\d+) pObj:(\S+) dObj:(\S+) pInfea\(1\):(\S+)")


def main():
    out = []
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
    with tempfile.TemporaryDirectory() as td:
        for name, flags in CASES:
            js = os.path.join(td, "o.json")
            r = subprocess.run([HARNESS, "solve", os.path.join(INST, f"{name}.dat-s"), *flags, "--jsonfile", js],
                               capture_output=True, text=True, cwd=td, env=env)
            res = {}
            for line in r.stdout.splitlines():
                if line.startswith("REF_RESULT"):
                    for kv in line.split()[1:]:
                        k, v = kv.split("=")
                        res[k] = float(v)
            log = [[int(a), int(b), float(c), float(d), float(e)] for a, b, c, d, e in LINE.findall(r.stdout)]
            out.append({"instance": name, "flags": flags, "result": res, "alm_log": log, "json": json.load(open(js))})
            print(name, flags, {k: res.get(k) for k in ("alm_inner", "alm_pobj", "rank")})
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
