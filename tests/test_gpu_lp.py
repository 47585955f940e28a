"""LoRADS's LP cone (the SDPA block of negative size) on the device: the LP block as the
diagonal cone at rank 1 (lrs_problem.cpp build_problem), its ADMM update the reference's
closed-form column sweep (lrs_kernels.hip k_lp_admm).

Reference side (the reference LoRADS C code built here, oracle/_ref; scripts/make_golden_lp.py,
scripts/make_golden_steps.py):
  tests/golden/steps_mc_lp60.npz        K trips of the inner loop (covered by test_gpu_steps.py)
  tests/golden/admm_sweep_lp_mc_lp60.npz  LORADSUpdateSDPLPVar + LORADSUpdateDualVar on seeded U, V, lambda
  tests/golden/solves_lp.json           whole solves of mc_lp60 and of the reference's bundled shmup4

Bars (per assertion): the sweep's U, V, lambda within 1e-6 (the SDP cone's CG at cg_tol 1e-9,
as tests/test_gpu_small_cg.py) and the LP block's values alone within 1e-6; whole mc_lp60 solve
reproduced step for step like the MaxCut solves (ALM inner +-2, objectives 1e-6, ADMM +-1);
shmup4 (thousands of L-BFGS steps through 3 cones: trajectories diverge under FP64 summation
order) within 10x the two certified gaps of the reference's objective, pinf <= 1e-4, same final
SDP rank."""
import importlib
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, ROOT, instance, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


def lp_data(path):
    """(c, {col: [(con, a)]}) of the LP block straight from the SDPA text (C = -F0)."""
    with open(path) as f:
        lines = [ln for ln in f if ln.strip() and ln.lstrip()[0] not in '*"']
    nb = int(lines[1].split()[0])
    dims = [int(x) for x in lines[2].replace(",", " ").split()[:nb]]
    lpb, nlp = nb, -dims[-1]
    c = np.zeros(nlp)
    cols = {}
    for ln in lines[4:]:
        t = ln.split()
        if len(t) != 5:
            continue
        con, blk, i, v = int(t[0]), int(t[1]), int(t[2]), float(t[4])
        if blk != lpb:
            continue
        if con == 0:
            c[i - 1] += -v
        else:
            cols.setdefault(i - 1, []).append((con - 1, v))
    return c, cols


def test_lp_sweep_matches_reference(solver_mod):
    """One ADMM sweep through the C-ABI operators: the SDP cone's two CG half-steps, then the LP
    cone's column sweep (lrs_op_admm_half(ctx, lp_cone, 0, ...): u_j and v_j of every column in
    column order), then the dual update -- against LORADSUpdateSDPLPVar + LORADSUpdateDualVar."""
    g = np.load(os.path.join(GOLDEN, "admm_sweep_lp_mc_lp60.npz"))
    rank, m = int(g["rank"]), int(g["m"])
    dims = [int(d) for d in g["dims"]]
    rho, tol = float(g["rho"]), float(g["cg_tol"])
    sv = solver_mod.Solver(instance("mc_lp60"))
    assert sv.dims == dims
    sv.set_rank([rank, 1])
    sv.set_factor(solver_mod.U, g["U0"])
    sv.set_factor(solver_mod.V, g["V0"])
    sv.set_vec(solver_mod.LAMBDA, g["lam0"])
    sv.admm_constr()
    for side in (0, 1):
        sv.admm_half(rho, tol, cone=0, side=side, init=False)
    sv.admm_half(rho, tol, cone=1, side=0, init=False)
    with pytest.raises(RuntimeError):
        sv.admm_half(rho, tol, cone=1, side=1, init=False)   # the sweep updates U and V together
    sv.dual_update(rho)
    U, V, lam = sv.get_factor(solver_mod.U), sv.get_factor(solver_mod.V), sv.get_vec(solver_mod.LAMBDA)
    nsdp = dims[0] * rank
    for key, ours in (("U", U), ("V", V), ("lam", lam)):
        assert rel_err(ours, g[key]) < 1e-6, (key, rel_err(ours, g[key]))
    for key, ours in (("U", U), ("V", V)):
        e = rel_err(ours[nsdp:], g[key][nsdp:])
        assert e < 1e-6, (key, "LP block", e)
    sv.close()


def _solves():
    with open(os.path.join(GOLDEN, "solves_lp.json")) as f:
        return {s["instance"]: s for s in json.load(f)}


def test_lp_solve_matches_reference(solver_mod):
    """mc_lp60 (a 60-row MaxCut with its diagonal constraints as inequalities through LP slacks,
    a free LP variable split in two and a dense LP column) solved whole: the reference's
    trajectory step for step."""
    ref = _solves()["mc_lp60"]
    rr = ref["result"]
    sv = solver_mod.Solver(instance("mc_lp60"))
    res = sv.solve(reoptLevel=0)
    assert abs(res["alm_inner"] - rr["alm_inner"]) <= 2, (res["alm_inner"], rr["alm_inner"])
    assert abs(res["alm_pobj"] - rr["alm_pobj"]) <= 1e-6 * abs(rr["alm_pobj"])
    assert abs(res["alm_dobj"] - rr["alm_dobj"]) <= 1e-6 * abs(rr["alm_dobj"])
    assert abs(res["admm_iter"] - rr["admm_iter"]) <= 1, (res["admm_iter"], rr["admm_iter"])
    assert abs(res["pobj"] - rr["admm_pobj"]) <= 1e-6 * abs(rr["admm_pobj"])
    assert abs(res["dobj"] - rr["admm_dobj"]) <= 1e-6 * abs(rr["admm_dobj"])
    # curr_rank counts the SDP cone only (the reference's rankElem); the LP cone stays at rank 1
    assert res["final_rank"] == int(rr["rank"])
    assert sv.get_rank()[1] == 1
    # the LP block's dual infeasibility part: per column c_j - sum_i lambda_i a_ij
    c, cols = lp_data(instance("mc_lp60"))
    lam = sv.get_vec(solver_mod.LAMBDA)
    s = c.copy()
    for j, ents in cols.items():
        for i, a in ents:
            s[j] += -lam[i] * a
    _, lmin = sv.dual_infeasibility()
    assert abs(lmin[1] - s.min()) <= 1e-9 * max(1.0, abs(s.min())), (lmin[1], s.min())
    sv.close()


def test_shmup4_solves_to_reference_objective(solver_mod):
    """The reference's own bundled shmup4 (two SDP blocks of 1 681 / 1 680 rows and an LP block of
    1 600 columns, m = 800) at --reoptLevel 0."""
    ref = _solves()["shmup4"]
    rr = ref["result"]
    sv = solver_mod.Solver(os.path.join(ROOT, "data", "bundled", "shmup4.dat-s"))
    res = sv.solve(reoptLevel=0)
    sv.close()
    tol = 10 * (res["gap"] + rr["admm_gap"]) + 1e-6
    assert abs(res["pobj"] - rr["admm_pobj"]) <= tol * (1 + abs(rr["admm_pobj"])), (res["pobj"], rr["admm_pobj"], tol)
    assert res["pinf"] <= 1e-4
    print(f"shmup4: device pobj {res['pobj']:.8e} gap {res['gap']:.2e} in {res['solve_time']:.2f} s "
          f"(ALM {res['alm_inner']}, ADMM {res['admm_iter']}); reference {rr['admm_pobj']:.8e} gap "
          f"{rr['admm_gap']:.2e} in {rr['solve_time']:.1f} s")
