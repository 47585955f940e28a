"""Per-iteration parity of the FUSED ALM inner iteration against the reference.

tests/golden/steps_<name>.npz come from the reference LoRADS C code itself
(scripts/make_golden_steps.py -> oracle/ref_harness.c `alm_steps`): from the reference's
initial point, exactly K trips of the inner L-BFGS loop (lorads_alm.c:1302-1379, with the
dual / rho updates between inner loops of lorads_alm.c:1380-1409).  The device runs the
same K trips through its product kernels (Solver.alm_steps = lrs_solve with a phase-1
budget of K) on every kernel family:

  path 0  latency-regime kernels k_lat_a / k_lat_b (+ slice blocks and k_lat_f on hub rows)
  path 1  general row kernels k_it_a / (k_it_g) / k_it_b, fused (small-n regime)
  path 2  general row kernels in their bandwidth-regime form (split launches)
  path 3  path 2 with the long-row neighbour kernels k_wide_a / k_wide_b

Tolerances: tau_k to 1e-9 relative with the same root count; R_K, G_K, A(R_K R_K^T),
the newest L-BFGS pair to 1e-9 relative (norm-wise; FP64 summation-order rounding grows
through K dependent trips); ||G||^2 and pinf to 1e-9.
"""
import importlib
import os

import numpy as np
import pytest

from golden_util import GOLDEN, ROOT, rel_err

pytestmark = pytest.mark.gpu
STEP_CASES = ["mc_rand200", "mc_torus12x10", "mc_rand300w", "theta40", "theta25x3", "rsparse60", "checker_1.5",
              "mc_rand300w_r290", "mc_lp60"]
# fixtures whose n x r arrays are stored as n x k projections V @ Omega (scripts/make_golden_steps.py)
PROJ = {"mc_rand300w_r290": 4}


def project(v, n, k, seed=7):
    r = v.size // n
    om = np.random.default_rng(seed).standard_normal((r, k))
    return v.reshape(r, n).T @ om
TOL = 1e-9


def _path(name):
    if name == "checker_1.5":
        return os.path.join(ROOT, "data", "bundled", "checker_1.5.dat-s")
    base = name[:name.rindex("_r")] if name in PROJ else name
    return os.path.join(GOLDEN, "instances", f"{base}.dat-s")


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


def _cases():
    out = []
    for name in STEP_CASES:
        for path in (0, 1, 2, 3):
            out.append((name, path))
    return out


@pytest.mark.parametrize("name,kpath", _cases())
def test_fused_iterations_match_reference(solver_mod, name, kpath, monkeypatch):
    monkeypatch.setenv("LRS_SMALL", "0")   # path 0 = the latency kernels here (path 4: below)
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    sv = solver_mod.Solver(_path(name))
    sv.set_kernel_path(kpath)
    worst = {}
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        d = sv.alm_steps(K, **kw)
        assert d["inner"] == K, (K, d["inner"])
        tau, rn, lag, pinf = trips[K - 1]
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
        assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)
        assert abs(d["beta"] - z[f"K{K}_beta"][0]) <= TOL * abs(z[f"K{K}_beta"][0])
        for key, ref in (("R", "R"), ("G", "G"), ("cvs", "cvs"), ("s", "s"), ("y", "y")):
            ours = d[key]
            if name in PROJ and key != "cvs":
                ours = project(ours, int(z["dims"][0]), PROJ[name])
            e = rel_err(ours, z[f"K{K}_{ref}"])
            worst[key] = max(worst.get(key, 0.0), e)
            assert e < TOL, (K, key, e)
        assert rel_err(d["lam"], z[f"K{K}_lam"]) < TOL or np.linalg.norm(z[f"K{K}_lam"]) == 0
        if kpath == 0 and name != "rsparse60":
            # the latency kernels are the ones that ran (rsparse60's multi-slot rows may not fit them)
            assert sv.kernel_path() in (0, 1)
        if kpath >= 1:
            assert sv.kernel_path() == 1
    print(f"{name} path {kpath}: worst rel errors {worst}")
    sv.close()


def test_budget_hook_resumes_same_solve(solver_mod):
    """W warmup trips + K timed trips through lrs_set_budget_hook == W + K trips in one go
    (bit for bit): the bench's timed region continues the same solve."""
    name = "mc_torus12x10"
    sv = solver_mod.Solver(_path(name))
    calls = []
    out = sv.alm_timed(7, 23, on_start=lambda: calls.append("start"), on_stop=lambda: calls.append("stop"),
                       reoptLevel=0)
    assert calls == ["start", "stop"] and out["done"] == 23 and out["inner"] == 30
    sv.ranks = sv.get_rank()
    R1 = sv.get_factor(solver_mod.R)
    d = sv.alm_steps(30, reoptLevel=0, phase1Tol=1e-300)
    assert np.array_equal(R1, d["R"])
    sv.close()

@pytest.mark.parametrize("name", STEP_CASES)
def test_fused_iterations_slot_tiles_match_reference(solver_mod, name, monkeypatch):
    """Path 3 with stage A's lower pattern in 2-D LDS tiles (k_tile_a, forced by
    LRS_SLOT_TILES=1 at load; C5-like cones take it by default): the same trips to 1e-9."""
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    sv = solver_mod.Solver(_path(name))
    sv.set_kernel_path(3)
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        d = sv.alm_steps(K, **kw)
        assert d["inner"] == K, (K, d["inner"])
        tau, rn, lag, pinf = trips[K - 1]
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
        for key in ("R", "G", "cvs", "s", "y"):
            ours = d[key]
            if name in PROJ and key != "cvs":
                ours = project(ours, int(z["dims"][0]), PROJ[name])
            assert rel_err(ours, z[f"K{K}_{key}"]) < TOL, (K, key)
    sv.close()


@pytest.mark.parametrize("name", ["mc_rand200_l3", "theta40_l3"])
def test_lbfgs_ring_of_three_matches_reference(solver_mod, name):
    """--lbfgsListLength 3 (data/lorads_solver.c:686-706: a ring of L pairs; LBFGSDirection's
    two-loop over min(innerIter, L) of them, lorads_alm.c:468-505): the reference's own trips
    (scripts/make_golden_steps.py with the flag) against run_inner_generic's, 1e-9."""
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    assert int(z["lbfgs_len"]) == 3
    base = name[:name.rindex("_l")]
    sv = solver_mod.Solver(os.path.join(GOLDEN, "instances", f"{base}.dat-s"))
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        d = sv.alm_steps(K, reoptLevel=0, lbfgsListLength=3)
        assert d["inner"] == K, (K, d["inner"])
        tau, rn, lag, pinf = trips[K - 1]
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
        assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)
        assert abs(d["beta"] - z[f"K{K}_beta"][0]) <= TOL * abs(z[f"K{K}_beta"][0])
        for key in ("R", "G", "cvs", "s", "y"):
            assert rel_err(d[key], z[f"K{K}_{key}"]) < TOL, (K, key)
    # a whole solve with the ring of 3 converges like the reference's default (objective within
    # the golden solve's certified gap)
    r = sv.solve(reoptLevel=0, lbfgsListLength=3)
    sv.close()
    assert r["pinf"] <= 1e-4 and r["alm_inner"] > 0


def test_lbfgs_ring_of_one(solver_mod):
    """--lbfgsListLength 1 (the reference itself crashes on it: its ring links are only set while
    adding nodes 2..L, data/lorads_solver.c:686-706): the generic ring path with one pair; the ALM
    phase converges to the L = 2 objective within both phases' certified gaps.  (When the ALM phase
    already meets phase2Tol the ADMM phase returns at once and reports the initial 1e30
    objective, as the reference's LORADSADMMOptimize / LORADSInitADMMState do.)"""
    a = solver_mod.Solver(os.path.join(GOLDEN, "instances", "mc_rand200.dat-s"))
    r1 = a.solve(reoptLevel=0, lbfgsListLength=1)
    r2 = a.solve(reoptLevel=0)
    a.close()
    tol = 10 * (r1["alm_gap"] + r2["alm_gap"]) + 1e-6
    assert abs(r1["alm_pobj"] - r2["alm_pobj"]) <= tol * abs(r2["alm_pobj"]), (r1["alm_pobj"], r2["alm_pobj"], tol)
    assert r1["alm_pinf"] <= 1e-3 and r1["alm_inner"] > 0


SMALL_CASES = [(n, c, "0") for n in ["mc_rand200", "mc_torus12x10", "mc_rand300w", "theta40", "theta25x3", "rsparse60"]
               for c in (["0", "1"] if n.startswith("theta") else ["0"])] + [("theta25x3", c, "1") for c in ("0", "1")]


@pytest.mark.parametrize("name,const,mc", SMALL_CASES)
def test_single_workgroup_inner_loop_matches_reference(solver_mod, name, const, mc, monkeypatch):
    """Kernel path 4: the whole inner loop of each run_inner call in one launch of one workgroup
    (lrs_kernels.hip k_small_alm; R and D in LDS, barriers between the trips' phases), theta's
    C = -J as a slot pattern (LRS_CONST_C=0) and as the constant objective's column sums (=1):
    the reference's own trips, 1e-9 as the multi-launch kernels.  mc = 1 (LRS_SMALL_MC): one
    workgroup per cone (theta25x3's three cones), the trips' sums exchanged between them."""
    monkeypatch.setenv("LRS_CONST_C", const)
    monkeypatch.setenv("LRS_SMALL_MC", mc)
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    sv = solver_mod.Solver(_path(name))
    sv.set_kernel_path(4)
    worst = {}
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        d = sv.alm_steps(K, **kw)
        assert sv.kernel_path() == 4
        assert d["inner"] == K, (K, d["inner"])
        tau, rn, lag, pinf = trips[K - 1]
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
        assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)
        assert abs(d["beta"] - z[f"K{K}_beta"][0]) <= TOL * abs(z[f"K{K}_beta"][0])
        for key in ("R", "G", "cvs", "s", "y"):
            e = rel_err(d[key], z[f"K{K}_{key}"])
            worst[key] = max(worst.get(key, 0.0), e)
            assert e < TOL, (K, key, e)
        assert rel_err(d["lam"], z[f"K{K}_lam"]) < TOL or np.linalg.norm(z[f"K{K}_lam"]) == 0
    print(f"{name} const {const}: worst rel errors {worst}")
    sv.close()


@pytest.mark.parametrize("name", ["theta40", "theta25x3", "mc_torus12x10"])
def test_single_workgroup_solve_matches_default(solver_mod, name, monkeypatch):
    """Whole solves on kernel path 4 against the default kernels (same bar as the golden solves:
    MaxCut objectives 1e-6, theta within the certified gaps)."""
    out = []
    for path, const in ((0, "0"), (4, "1")):
        monkeypatch.setenv("LRS_CONST_C", const)
        sv = solver_mod.Solver(_path(name))
        sv.set_kernel_path(path)
        out.append(sv.solve(reoptLevel=0))
        sv.close()
    a, b = out
    if name.startswith("mc_"):
        assert abs(a["alm_inner"] - b["alm_inner"]) <= 2
        for k in ("alm_pobj", "pobj"):
            assert abs(a[k] - b[k]) <= 1e-6 * abs(a[k]), (k, a[k], b[k])
    else:
        tol = 10 * (a["gap"] + b["gap"]) + 1e-6
        for k in ("pobj", "dobj"):
            assert abs(a[k] - b[k]) <= tol * (1 + abs(a[k])), (k, a[k], b[k], tol)
        assert b["pinf"] <= 1e-4


def test_one_workgroup_per_cone_timeout_falls_back(solver_mod, monkeypatch):
    """the one-workgroup-per-cone inner loop assumes its workgroups are co-resident; an
    exchange that times out (forced here: LRS_XWG_SPIN=-1, no waiting at all) must not end
    the solve nor leave a half-updated iterate -- the call is rerun from the state kept before the
    launch on the multi-launch iteration, and the trips still equal the reference's at 1e-9."""
    monkeypatch.setenv("LRS_SMALL_MC", "1")
    monkeypatch.setenv("LRS_XWG_SPIN", "-1")
    z = np.load(os.path.join(GOLDEN, "steps_theta25x3.npz"))
    sv = solver_mod.Solver(_path("theta25x3"))
    sv.set_kernel_path(4)
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        d = sv.alm_steps(K, reoptLevel=0)
        assert d["inner"] == K, (K, d["inner"])
        tau, rn, lag, pinf = trips[K - 1]
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
        for key in ("R", "G", "cvs", "s", "y"):
            assert rel_err(d[key], z[f"K{K}_{key}"]) < TOL, (K, key)
    assert sv.xwg_fallbacks() >= 1
    # the whole solve also completes (ALM, ADMM) on the fallback path
    res = sv.solve(reoptLevel=0)
    assert res["pinf"] <= 1e-4
    sv.close()
