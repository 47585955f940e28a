#!/usr/bin/env python3
"""Device-side look at the reference's tight solves (tests/golden/solves_tight.json and the
reference's final iterates tests/golden/tight_final_<name>.npz): the reference's final (R,
lambda) evaluated by the device operators (lrs_op_dimacs, lrs_op_dual_infeasibility) beside
the device's own solve at the same flags.  One JSON line per instance."""
import importlib
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
gold = {(g["instance"], g["flags"][-1]): g for g in json.load(open(os.path.join(ROOT, "tests", "golden",
                                                                                "solves_tight.json")))}
args = [a for a in sys.argv[1:] if not a.startswith("--")]
names = args or ["checker_1.5", "ice_2.0", "p_auss2_3.0", "theta3"]
LEVEL2 = "--level2" in sys.argv   # also a device solve at reoptLevel 2 (dual-infeasibility driven)
td = tempfile.mkdtemp()
for name in names:
    g = gold[(name, "1e-8")]
    path = os.path.join(ROOT, "data", "bundled", f"{name}.dat-s") if g["kind"] == "bundled" else \
        inst.config_instance(name, td)
    kw = {}
    fl = g["flags"]
    for q in range(0, len(fl), 2):
        k = fl[q].lstrip("-")
        kw[k] = int(fl[q + 1]) if k in ("reoptLevel", "fixedRank") else float(fl[q + 1])
    out = {"instance": name, "ref": {k: g["result"][k] for k in ("admm_pobj", "admm_dobj", "admm_pinf", "admm_gap")}}
    z = np.load(os.path.join(ROOT, "tests", "golden", f"tight_final_{name}.npz"))
    sv = solver.Solver(path)
    sv.set_rank([int(r) for r in z["ranks"]])
    sv.set_factor(solver.R, z["R"])
    sv.set_vec(solver.LAMBDA, z["lam"])
    out["ref_iterate_on_device"] = sv.dimacs()
    l1, lmin = sv.dual_infeasibility()
    out["ref_iterate_on_device"].update({"dinf": l1, "lambda_min": list(map(float, np.atleast_1d(lmin)))})
    out["ref_rank"] = [int(r) for r in z["ranks"]]
    r = sv.solve(**kw)
    out["device"] = {k: r[k] for k in ("pobj", "dobj", "pinf", "gap", "dinf", "final_rank", "alm_inner", "admm_iter",
                                       "status", "solve_time")}
    out["rel_pobj"] = abs(r["pobj"] - g["result"]["admm_pobj"]) / abs(g["result"]["admm_pobj"])
    l1, lmin = sv.dual_infeasibility()
    out["device"]["lambda_min"] = list(map(float, np.atleast_1d(lmin)))
    out["device"]["trace_X"] = float(np.sum(sv.get_factor(solver.R) ** 2))
    if LEVEL2:
        kw2 = dict(kw, reoptLevel=2)
        r2 = sv.solve(**kw2)
        l1, lmin = sv.dual_infeasibility()
        out["device_level2"] = {k: r2[k] for k in ("pobj", "dobj", "pinf", "gap", "dinf", "final_rank", "alm_inner",
                                                   "admm_iter", "status", "solve_time")}
        out["device_level2"]["lambda_min"] = list(map(float, np.atleast_1d(lmin)))
        out["device_level2"]["trace_X"] = float(np.sum(sv.get_factor(solver.R) ** 2))
    sv.close()
    print(json.dumps(out), flush=True)
