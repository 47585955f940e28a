#!/usr/bin/env python3
"""The reference's final iterates (R per cone, lambda) of the theta configs of
tests/golden/solves_configs.json, for the certified-interval test of tests/test_gpu_configs.py:
the same instances and flags as scripts/make_golden_configs.py, solved by the reference C code
built under oracle/_ref with REF_DUMP (oracle/ref_harness.c), saved as
tests/golden/configs_final_<name>.npz.  The run's primal objective must equal the golden one
(the same deterministic solve).  CPU only; needs /root/reference.
Run:  python scripts/make_golden_configs_final.py"""
import importlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from make_golden_bundled import save_final   # noqa: E402
from make_golden_configs import HARNESS, SDPLIB   # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "solves_configs.json")


def main():
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    gold = {g["config"]: g for g in json.load(open(GOLD))}
    with tempfile.TemporaryDirectory() as td:
        for name in ("theta3", "theta3x3"):
            path = inst.config_instance(name, td)
            dump = os.path.join(td, name + ".final")
            env = dict(os.environ, OPENBLAS_NUM_THREADS="1", REF_DUMP=dump)
            r = subprocess.run([HARNESS, "solve", path, *SDPLIB], capture_output=True, text=True, cwd=td, env=env)
            res = {}
            for line in r.stdout.splitlines():
                if line.startswith("REF_RESULT"):
                    for kv in line.split()[1:]:
                        k, v = kv.split("=")
                        res[k] = float(v)
            assert res.get("admm_pobj") == gold[name]["result"]["admm_pobj"], (name, res, gold[name]["result"])
            save_final(dump, os.path.join(ROOT, "tests", "golden", f"configs_final_{name}.npz"))
            print(name, res.get("admm_pobj"), flush=True)


if __name__ == "__main__":
    main()
