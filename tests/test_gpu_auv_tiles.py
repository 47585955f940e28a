"""A(X Y^T) over 2-D LDS tiles (k_auv_tile + k_auv_tsum, lrs_kernels.hip) against the
per-entry gather k_auv_con and the reference's golden vectors (MI355X).

The tiled path is taken for cones whose lower-triangle tiles hold >= kAuvMinPerTile entries on average at
n >= kAuvMinN (C5-like), or always with LRS_AUV_TILES=1 (read when the problem is
uploaded).  Reference semantics: coneAUV data/lorads_sdp_conic.c:378-385 and
LORADSUpdateConstrValCG lorads_admm.c:442-459.  Tolerances: the entry dot products are
summed in another order than the gather's lane-group tree, so 1e-10 relative against the
reference (as test_gpu_parity.py) and 1e-12 against the gather path."""
import importlib

import numpy as np
import pytest

from golden_util import KERNEL_CASES, instance, load_kernels, rel_err, split_inputs

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


@pytest.mark.parametrize("name", KERNEL_CASES)
def test_tiled_auut_and_cg_match_reference(solver_mod, name, monkeypatch):
    monkeypatch.setenv("LRS_AUV_TILES", "1")
    g = load_kernels(name)
    s = split_inputs(g)
    sv = solver_mod.Solver(instance(name))
    sv.set_rank([s["rank"]] * len(s["dims"]))
    sv.set_factor(solver_mod.R, s["R"])
    sv.time_auut(1)                                   # A(R R^T), MODE 1
    assert rel_err(sv.get_vec(solver_mod.Q1), g["cvs_rr"]) < TOL
    # ADMM half step: the CG's A(sym(p V^T)) and the right-hand side's A(U V^T) (MODE 0)
    sv.set_factor(solver_mod.U, s["U"])
    sv.set_factor(solver_mod.V, s["V"])
    sv.set_vec(solver_mod.LAMBDA, s["lam"])
    u, rhs, it = sv.admm_half(s["rho_admm"], s["cg_tol"])
    assert rel_err(rhs, g["rhs_cg"]) < TOL
    assert rel_err(u, g["u_cg"]) < 1e-6
    assert abs(it - g["cg_iters"]) <= max(2, 0.1 * g["cg_iters"])
    sv.close()


def _c5_like(solver_mod, tiles, monkeypatch, n=3000, m=40000, r=24):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    monkeypatch.setenv("LRS_AUV_TILES", tiles)
    sv = solver_mod.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(n, m, 6, 11)))
    sv.set_rank([r])
    return sv


def test_tiled_auut_matches_gather_at_scale(solver_mod, monkeypatch):
    """n = 3000, m = 4e4, 6 entries per constraint (ragged last tiles: 3000 = 23 x 128 + 56;
    r = 24 < kAuvC: a partial column chunk), both modes, against the per-entry gather."""
    rng = np.random.default_rng(5)
    n, r = 3000, 24
    R = rng.standard_normal(n * r)
    U = rng.standard_normal(n * r)
    V = rng.standard_normal(n * r)
    lam = rng.standard_normal(40000)
    out = {}
    for tiles in ("0", "1"):
        sv = _c5_like(solver_mod, tiles, monkeypatch)
        sv.set_factor(solver_mod.R, R)
        sv.time_auut(1)
        q = sv.get_vec(solver_mod.Q1)
        sv.set_factor(solver_mod.U, U)
        sv.set_factor(solver_mod.V, V)
        sv.set_vec(solver_mod.LAMBDA, lam)
        u, rhs, it = sv.admm_half(2.0, 1e-8, 60)
        out[tiles] = (q, u, rhs, it)
        sv.close()
    (q0, u0, rhs0, it0), (q1, u1, rhs1, it1) = out["0"], out["1"]
    assert rel_err(q1, q0) < 1e-12
    assert rel_err(rhs1, rhs0) < 1e-12
    assert abs(it1 - it0) <= 1
    assert rel_err(u1, u0) < 1e-8


def test_tiled_path_whole_solve(solver_mod, monkeypatch):
    """A bounded ALM phase + ADMM on a C5-like problem: the tiled A(.) (default at this size)
    and the per-entry gather give the same trajectory to rounding."""
    res = {}
    for tiles in ("0", "1"):
        sv = _c5_like(solver_mod, tiles, monkeypatch, n=2500, m=30000)
        res[tiles] = sv.solve(fixedRank=16, reoptLevel=0, almInnerBudget=200, maxADMMIter=30)
        sv.close()
    a, b = res["0"], res["1"]
    assert a["alm_inner"] == b["alm_inner"]
    assert abs(a["admm_iter"] - b["admm_iter"]) <= 1
    assert abs(a["alm_pobj"] - b["alm_pobj"]) <= 1e-9 * max(1.0, abs(a["alm_pobj"]))
    assert abs(a["pobj"] - b["pobj"]) <= 1e-6 * max(1.0, abs(a["pobj"]))


@pytest.mark.parametrize("name", KERNEL_CASES)
def test_tiled_pattern_sddmm_matches_reference(solver_mod, name, monkeypatch):
    """The pattern SDDMM (lrs_op_q12's sym(R D^T) / D D^T, lrs_op_constr_rr's R R^T and their
    <C, .> sums) and the SpMM (gradient, ADMM half step) over the slot tiles (LRS_SLOT_TILES=1; C5-like cones by default) against the
    reference's ALMCalq12p12 / primalInfeasibility / CalObjRR vectors at 1e-10."""
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    g = load_kernels(name)
    s = split_inputs(g)
    sv = solver_mod.Solver(instance(name))
    sv.set_rank([s["rank"]] * len(s["dims"]))
    sv.set_factor(solver_mod.R, s["R"])
    sv.set_factor(solver_mod.D, s["D"])
    q1, p1, q2, p2 = sv.q12()
    assert rel_err(q1, g["q1"]) < TOL and rel_err(q2, g["q2"]) < TOL
    assert abs(p1 - g["p1"]) <= TOL * max(1, abs(g["p1"])) and abs(p2 - g["p2"]) <= TOL * max(1, abs(g["p2"]))
    cvs, pinf, pobj = sv.constr_rr()
    assert rel_err(cvs, g["cvs_rr"]) < TOL
    assert abs(pinf - g["pinf_rr"]) <= TOL * max(1, abs(g["pinf_rr"]))
    assert abs(pobj - g["pobj_rr"]) <= TOL * max(1, abs(g["pobj_rr"]))
    # ALMCalGrad and the ADMM half step: S R / S Y over the tiles (launch_spmm -> k_tile_b2 +
    # k_spmm_fin)
    sv.set_vec(solver_mod.LAMBDA, s["lam"])
    sv.set_vec(solver_mod.CVS, s["cvs"])
    G, lag = sv.grad(s["rho"])
    assert rel_err(G, g["grad"]) < TOL
    assert abs(lag - g["lag"]) <= TOL * g["lag"]
    sv.set_factor(solver_mod.U, s["U"])
    sv.set_factor(solver_mod.V, s["V"])
    sv.set_vec(solver_mod.LAMBDA, s["lam"])
    u, rhs, it = sv.admm_half(s["rho_admm"], s["cg_tol"])
    assert rel_err(rhs, g["rhs_cg"]) < TOL
    assert rel_err(u, g["u_cg"]) < 1e-6
    assert abs(it - g["cg_iters"]) <= max(2, 0.1 * g["cg_iters"])
    sv.close()
