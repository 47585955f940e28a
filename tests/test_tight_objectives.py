"""Objectives pinned beyond the default stopping rule.

At the reference's default phase2Tol 1e-5 (main.c:75) the general SDPs it ships (checker_1.5,
ice_2.0, p_auss2_3.0) stop primal-dual optimal on both sides with primal objectives ~1e-4 apart
(tests/test_bundled.py): the stopping rule fixes them no closer.  Solved to phase2Tol 1e-7 and
1e-8 by the reference itself (tests/golden/solves_tight.json, scripts/make_golden_tight.py, the
reference C code built under oracle/_ref), its primal and dual objectives close to ~1e-8 of each
other -- the optimum.  The device solves the same files with the same flags; its primal objective
must then agree with the reference's to 1e-6 relative (north_star's objective bar), i.e. both
sides converge to the same optimum when pushed, and the 1e-4 spread at 1e-5 is the stopping
rule's, not a different limit point.  theta3 (SDPLIB flags) stops there on the reference's side
at a gap of ~4e-7 (its ADMM exits on the relaxed test of main.c:540): the bar is 10x the two
certified gaps there, as for the other theta-class whole solves."""
import importlib
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "solves_tight.json")
DATA = os.path.join(ROOT, "data", "bundled")
GENERAL = ["checker_1.5", "ice_2.0", "p_auss2_3.0"]
OBJ_TOL = 1e-6


def golden():
    with open(GOLD) as f:
        return {(g["instance"], g["flags"][-1]): g for g in json.load(f)}


def kwargs_of(flags):
    kw = {}
    for q in range(0, len(flags), 2):
        k = flags[q].lstrip("-")
        kw[k] = int(flags[q + 1]) if k in ("reoptLevel", "fixedRank") else float(flags[q + 1])
    return kw


def test_tight_fixtures_converged():
    """The reference's own tight solves: primal-dual optimal at the tightened tolerance, the
    objectives' spread shrinking with it (so they pin the optimum, not a stopping point)."""
    g = golden()
    for name in GENERAL:
        for tol in ("1e-7", "1e-8"):
            r = g[(name, tol)]["result"]
            assert r["admm_pinf"] <= float(tol) and r["admm_gap"] <= 5 * float(tol), (name, tol, r)
        a, b = g[(name, "1e-7")]["result"], g[(name, "1e-8")]["result"]
        # the 1e-8 objective within the 1e-7 run's certified neighbourhood
        assert abs(a["admm_pobj"] - b["admm_pobj"]) <= 1e-5 * abs(b["admm_pobj"]), (name, a, b)
        assert abs(b["admm_pobj"] - b["admm_dobj"]) <= 1e-7 * abs(b["admm_pobj"]), (name, b)
    assert ("theta3", "1e-8") in g


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


@pytest.mark.gpu
@pytest.mark.parametrize("name", GENERAL)
def test_general_sdp_objective_at_1e8_matches_reference(solver_mod, name):
    g = golden()[(name, "1e-8")]
    ref = g["result"]
    sv = solver_mod.Solver(os.path.join(DATA, f"{name}.dat-s"))
    r = sv.solve(**kwargs_of(g["flags"]))
    sv.close()
    rel = abs(r["pobj"] - ref["admm_pobj"]) / abs(ref["admm_pobj"])
    print(f"{name}: device pobj {r['pobj']:.12g} dobj {r['dobj']:.12g} gap {r['gap']:.2e} pinf {r['pinf']:.2e}; "
          f"reference pobj {ref['admm_pobj']:.12g} dobj {ref['admm_dobj']:.12g}; rel {rel:.2e}")
    assert r["pinf"] <= 1e-8 and r["gap"] <= 5e-8, r
    assert rel <= OBJ_TOL, (r["pobj"], ref["admm_pobj"], rel)


@pytest.mark.gpu
def test_theta3_objective_at_1e8_matches_reference(solver_mod, tmp_path):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    g = golden()[("theta3", "1e-8")]
    ref = g["result"]
    path = inst.config_instance("theta3", str(tmp_path))
    sv = solver_mod.Solver(path)
    r = sv.solve(**kwargs_of(g["flags"]))
    sv.close()
    tol = 10 * (ref["admm_gap"] + r["gap"]) + 1e-7
    rel = abs(r["pobj"] - ref["admm_pobj"]) / abs(ref["admm_pobj"])
    print(f"theta3: device pobj {r['pobj']:.12g} gap {r['gap']:.2e}; reference {ref['admm_pobj']:.12g} "
          f"gap {ref['admm_gap']:.2e}; rel {rel:.2e} bar {tol:.2e}")
    assert rel <= tol, (r["pobj"], ref["admm_pobj"], rel, tol)
