"""The single-workgroup ADMM half-step (lrs_kernels.hip k_small_cg: LORADSUpdateSDPVarOne's
right-hand side, CGSolve and the cone's constraint refresh in one launch) against the
multi-launch device CG (LRS_SMALL_CG=0) and the reference's own sweep
(tests/golden/admm_sweep_*.npz, scripts/make_golden_admm.py), on the instances where it is
taken (every cone of <= 256 rows; theta with C = -J as slots and in the rank-one form)."""
import importlib
import os

import numpy as np
import pytest

from golden_util import instance

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


def rel(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def sweep(solver_mod, name, monkeypatch, small):
    """LORADSUpdateSDPVar over every cone + LORADSUpdateDualVar through the C-ABI operators."""
    monkeypatch.setenv("LRS_SMALL_CG", "1" if small else "0")
    k = np.load(os.path.join(ROOT, "tests", "golden", f"kernels_{name}.npz"))
    vec, m, rank = k["inputs"], int(k["m"]), int(k["rank"])
    dims = [int(d) for d in k["dims"]]
    NR = sum(d * rank for d in dims)
    tail = vec[9 * NR + 2 * m:]
    rho = float(tail[3])
    tol = float(np.load(os.path.join(ROOT, "tests", "golden", f"admm_sweep_{name}.npz"))["cg_tol"])
    sv = solver_mod.Solver(instance(name))
    sv.set_rank([rank] * len(dims))
    sv.set_factor(solver_mod.U, vec[7 * NR:8 * NR])
    sv.set_factor(solver_mod.V, vec[8 * NR:9 * NR])
    sv.set_vec(solver_mod.LAMBDA, vec[9 * NR:9 * NR + m])
    sv.admm_constr()
    its, rhs = [], []
    for c in range(len(dims)):
        for side in (0, 1):
            _, rh, it = sv.admm_half(rho, tol, cone=c, side=side, init=False)
            its.append(it)
            rhs.append(rh)
    sv.dual_update(rho)
    out = dict(U=sv.get_factor(solver_mod.U), V=sv.get_factor(solver_mod.V), lam=sv.get_vec(solver_mod.LAMBDA),
               its=np.array(its), rhs=rhs)
    sv.close()
    return out


@pytest.mark.parametrize("name", ["theta25x3", "theta40", "mc_rand200", "rsparse60"])
def test_small_cg_matches_multi_launch_and_reference(solver_mod, monkeypatch, name):
    a = sweep(solver_mod, name, monkeypatch, small=True)
    b = sweep(solver_mod, name, monkeypatch, small=False)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"admm_sweep_{name}.npz"))
    # the half-steps' right-hand sides: the same arithmetic in another summation order
    for x, y in zip(a["rhs"], b["rhs"]):
        assert rel(x, y) < 1e-10
    # CG solutions at cg_tol 1e-9: both paths and the reference within 1e-6 (the bar of the
    # single half-step test), the two device paths closer
    for key in ("U", "V", "lam"):
        assert rel(a[key], b[key]) < 1e-7, (key, rel(a[key], b[key]))
        assert rel(a[key], g[key]) < 1e-6, (key, rel(a[key], g[key]))
    # CG counts (hundreds here, rounding-sensitive near the tolerance): as tests/test_capi.py,
    # 50 % past the n r unknowns of a solve (there the count is set by rounding alone)
    k = np.load(os.path.join(ROOT, "tests", "golden", f"kernels_{name}.npz"))
    dims, rank = [int(d) for d in k["dims"]], int(k["rank"])
    for q, (x, y) in enumerate(zip(a["its"], b["its"])):
        bar = 0.5 if max(x, y) > dims[q // 2] * rank else 0.25
        assert abs(int(x) - int(y)) <= max(2, bar * y), (a["its"], b["its"])
    assert abs(a["its"].sum() - float(g["cg_total"])) <= max(4, 0.15 * float(g["cg_total"]))


@pytest.mark.parametrize("name,flags", [("theta40", dict(reoptLevel=0)), ("theta25x3", dict(reoptLevel=0))])
def test_small_cg_whole_solve(solver_mod, monkeypatch, name, flags):
    """Whole solves with the ADMM phase on the single-workgroup half-step against the multi-launch
    CG: the ALM phase is identical (the ADMM phase starts from the same point), ADMM iterations
    within 2 % and the objectives within 10 x the certified gaps, as the reference bars of
    tests/test_gpu_parity.py."""
    res = {}
    for small in (True, False):
        monkeypatch.setenv("LRS_SMALL_CG", "1" if small else "0")
        sv = solver_mod.Solver(instance(name))
        res[small] = sv.solve(**flags)
        sv.close()
    a, b = res[True], res[False]
    assert a["alm_inner"] == b["alm_inner"] and a["alm_pobj"] == b["alm_pobj"]
    assert abs(a["admm_iter"] - b["admm_iter"]) <= max(2, 0.02 * b["admm_iter"])
    tol = 10 * (a["gap"] + b["gap"]) + 1e-6
    assert abs(a["pobj"] - b["pobj"]) <= tol * (1 + abs(b["pobj"]))
    assert a["pinf"] <= 1e-4 and a["gap"] <= max(1e-4, 10 * b["gap"])


def _write_theta_cycle(path, n):
    """Lovasz theta of the n-cycle in SDPA form: min <-J, X> s.t. tr X = 1, X_ij = 0 on the edges."""
    edges = [(i, (i + 1) % n) for i in range(n)]
    m = 1 + len(edges)
    with open(path, "w") as f:
        f.write(f"{m}\n1\n{n}\n" + " ".join(["1.0"] + ["0.0"] * len(edges)) + "\n")
        for i in range(1, n + 1):
            for j in range(i, n + 1):
                f.write(f"0 1 {i} {j} 1.0\n")   # F0 = J, C = -F0
        for i in range(1, n + 1):
            f.write(f"1 1 {i} {i} 1.0\n")
        for c, (i, j) in enumerate(edges):
            a, b = min(i, j) + 1, max(i, j) + 1
            f.write(f"{c + 2} 1 {a} {b} 1.0\n")


def test_small_cg_tiny_cone_rank_below_16(solver_mod, monkeypatch, tmp_path):
    """A cone with r < 16 and a handful of constraints (theta of the 5-cycle: n = 5, m = 6, r = 3):
    the single-workgroup CG's 16-lane column groups read Y's row pitch past r (those
    lanes must read finite words -- Y's zeroed pad or a clamped in-row column -- never the LDS past
    the last row).  The half-steps match the multi-launch CG and stay finite."""
    path = str(tmp_path / "theta_c5.dat-s")
    _write_theta_cycle(path, 5)
    rng = np.random.default_rng(11)
    out = []
    for small in (True, False):
        monkeypatch.setenv("LRS_SMALL_CG", "1" if small else "0")
        sv = solver_mod.Solver(path)
        sv.set_rank([3])
        n = sv.nr()
        U0, V0 = rng.standard_normal(n), rng.standard_normal(n)
        lam = rng.standard_normal(sv.m)
        rng = np.random.default_rng(11)   # the same inputs for both runs
        sv.set_factor(solver_mod.U, U0)
        sv.set_factor(solver_mod.V, V0)
        sv.set_vec(solver_mod.LAMBDA, lam)
        sv.admm_constr()
        for side in (0, 1, 0, 1):
            sv.admm_half(2.0, 1e-10, cone=0, side=side, init=False)
        out.append((sv.get_factor(solver_mod.U), sv.get_factor(solver_mod.V)))
        sv.close()
    (ua, va), (ub, vb) = out
    assert np.all(np.isfinite(ua)) and np.all(np.isfinite(va))
    assert rel(ua, ub) < 1e-8 and rel(va, vb) < 1e-8, (rel(ua, ub), rel(va, vb))


def test_small_cg_cones_side_by_side_equal_the_sweep(solver_mod, monkeypatch):
    """theta25x3 (three cones, no constraint in two): every cone's half-step of one side in one
    launch (a block a cone, LRS_SMALL_CG_BATCH default) against the reference's cone-by-cone
    sweep (=0).  The cones' solves and refreshes touch disjoint rows and constraints, so the
    whole solve is bitwise the same."""
    res = {}
    for batch in ("1", "0"):
        monkeypatch.setenv("LRS_SMALL_CG_BATCH", batch)
        sv = solver_mod.Solver(instance("theta25x3"))
        res[batch] = sv.solve(reoptLevel=0)
        sv.close()
    a, b = res["1"], res["0"]
    assert a["admm_iter"] > 0
    for key in ("alm_inner", "admm_iter", "pobj", "dobj", "pinf", "gap", "cg_iter"):
        if key in a:
            assert a[key] == b[key], (key, a[key], b[key])


@pytest.mark.parametrize("name", ["theta25x3", "theta40", "mc_rand200"])
def test_small_eval_matches_operators(solver_mod, monkeypatch, name):
    """The ADMM iteration's evaluation of small cones in one launch (k_small_eval: R = (U + V) / 2,
    A(R R^T), the residual, <C, R R^T>, b^T lambda) against the operator launches
    (LRS_SMALL_EVAL=0: k_avg, the SDDMM, the gather, the dots) on the reference sweep's inputs:
    the same values up to summation order."""
    k = np.load(os.path.join(ROOT, "tests", "golden", f"kernels_{name}.npz"))
    vec, m, rank = k["inputs"], int(k["m"]), int(k["rank"])
    dims = [int(d) for d in k["dims"]]
    NR = sum(d * rank for d in dims)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("LRS_SMALL_EVAL", flag)
        sv = solver_mod.Solver(instance(name))
        sv.set_rank([rank] * len(dims))
        sv.set_factor(solver_mod.U, vec[7 * NR:8 * NR])
        sv.set_factor(solver_mod.V, vec[8 * NR:9 * NR])
        sv.set_vec(solver_mod.LAMBDA, vec[9 * NR:9 * NR + m])
        out[flag] = (sv.dimacs(admm=True), sv.get_factor(solver_mod.R), sv.get_vec(solver_mod.CVS))
        sv.close()
    (a, ra, ca), (b, rb, cb) = out["1"], out["0"]
    assert np.array_equal(ra, rb)
    assert rel(ca, cb) < 1e-13
    for key in ("pobj", "dobj"):
        assert abs(a[key] - b[key]) <= 1e-12 * max(1.0, abs(b[key])), (key, a[key], b[key])
    assert abs(a["pinf"] - b["pinf"]) <= 1e-10 * b["pinf"] + 1e-300, (a["pinf"], b["pinf"])
