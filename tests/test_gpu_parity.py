"""HIP path vs the reference's golden vectors and the CPU oracle (MI355X).

Every check goes through the C-ABI (include/lrsdp.h).  Tolerances: FP64 kernels
agree with the reference to summation-order rounding (1e-10 relative); whole
solves follow the rules of tests/test_oracle_golden.py."""
import importlib
import json
import os
import subprocess

import numpy as np
import pytest

from golden_util import KERNEL_CASES, instance, load_kernels, load_solves, rel_err, split_inputs

pytestmark = pytest.mark.gpu
TOL = 1e-10


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


@pytest.mark.parametrize("name", KERNEL_CASES)
def test_device_kernels_match_reference(solver_mod, name):
    g = load_kernels(name)
    s = split_inputs(g)
    sv = solver_mod.Solver(instance(name))
    sv.set_rank([s["rank"]] * len(s["dims"]))
    S = solver_mod
    # (1) ALMCalq12p12
    sv.set_factor(S.R, s["R"])
    sv.set_factor(S.D, s["D"])
    q1, p1, q2, p2 = sv.q12()
    assert rel_err(q1, g["q1"]) < TOL and rel_err(q2, g["q2"]) < TOL
    assert abs(p1 - g["p1"]) <= TOL * max(1, abs(g["p1"])) and abs(p2 - g["p2"]) <= TOL * max(1, abs(g["p2"]))
    # (2) primalInfeasibility + CalObjRR
    cvs, pinf, pobj = sv.constr_rr()
    assert rel_err(cvs, g["cvs_rr"]) < TOL
    assert abs(pinf - g["pinf_rr"]) <= TOL * max(1, abs(g["pinf_rr"]))
    assert abs(pobj - g["pobj_rr"]) <= TOL * max(1, abs(g["pobj_rr"]))
    # (3) ALMCalGrad
    sv.set_vec(S.LAMBDA, s["lam"])
    sv.set_vec(S.CVS, s["cvs"])
    G, lag = sv.grad(s["rho"])
    assert rel_err(G, g["grad"]) < TOL
    assert abs(lag - g["lag"]) <= TOL * g["lag"]
    # (4) ALMLineSearch on (R, D) with q0 = b - cvs
    sv.q12()
    tau, rn = sv.line_search(s["rho"])
    assert rn == int(g["rootnum"])
    assert abs(tau - g["tau"]) <= 1e-9 * max(1, abs(g["tau"]))
    # (5) L-BFGS two-loop (NodeNum 2 and 1) + UseGrad
    sv.set_factor(S.G, s["G"])
    sv.set_factor(S.S0, s["s1"]); sv.set_factor(S.Y0, s["y1"])
    sv.set_factor(S.S1, s["s2"]); sv.set_factor(S.Y1, s["y2"])
    d2 = sv.lbfgs(2, s["beta1"], s["beta2"])
    assert rel_err(d2, g["d_lbfgs2"]) < 1e-9
    d1 = sv.lbfgs(1, s["beta1"], s["beta2"])
    assert rel_err(d1, g["d_lbfgs1"]) < 1e-9
    # (6) ADMM half step (CG)
    sv.set_factor(S.U, s["U"]); sv.set_factor(S.V, s["V"])
    sv.set_vec(S.LAMBDA, s["lam"])
    u, rhs, it = sv.admm_half(s["rho_admm"], s["cg_tol"])
    assert rel_err(rhs, g["rhs_cg"]) < TOL
    assert rel_err(u, g["u_cg"]) < 1e-6
    assert abs(it - g["cg_iters"]) <= max(2, 0.1 * g["cg_iters"])
    sv.close()


@pytest.mark.parametrize("case", range(7))
def test_device_solve_matches_reference(solver_mod, case):
    s = load_solves()[case]
    flags = s["flags"]
    kw = {}
    for k, v in zip(flags[0::2], flags[1::2]):
        k = k.lstrip("-")
        kw[k] = int(v) if k in ("reoptLevel", "fixedRank") else float(v)
    sv = solver_mod.Solver(instance(s["instance"]))
    res = sv.solve(**kw)
    r = s["result"]
    # final_rank is the sum over cones (lorads_sum_rank, lorads_logging.c:199-213);
    # REF_RESULT rank is cone 0's only
    assert res["final_rank"] == s["json"]["trajectory"]["phase_1"]["curr_rank"][-1]
    if s["instance"].startswith("mc_"):
        assert abs(res["alm_inner"] - r["alm_inner"]) <= max(2, 0.02 * r["alm_inner"])
        for ours, ref in (("alm_pobj", "alm_pobj"), ("alm_dobj", "alm_dobj"), ("pobj", "admm_pobj")):
            assert abs(res[ours] - r[ref]) <= 1e-6 * max(1.0, abs(r[ref])), (ours, res[ours], r[ref])
    else:
        tol = 10 * (r["admm_gap"] + res["gap"]) + 1e-6
        for ours, ref in (("pobj", "admm_pobj"), ("dobj", "admm_dobj")):
            assert abs(res[ours] - r[ref]) <= tol * (1 + abs(r[ref])), (ours, res[ours], r[ref], tol)
        assert res["pinf"] <= 1e-4
    sv.close()


def test_cli_drop_in_json(solver_mod, tmp_path):
    out = tmp_path / "o.json"
    ok, t, pobj = solver_mod.run_lorads(instance("mc_rand200"), out, {"reoptLevel": "0", "phase1Tol": "1e-2",
                                                                       "heuristicFactor": "10"})
    assert ok and t > 0
    ref = [s for s in load_solves() if s["instance"] == "mc_rand200" and "--phase1Tol" in s["flags"]][0]
    assert abs(pobj - ref["json"]["metrics"]["primal_obj"]) <= 1e-6 * abs(ref["json"]["metrics"]["primal_obj"])
    js = json.load(open(out))
    assert set(js["metrics"]) == set(ref["json"]["metrics"])
    assert set(js["trajectory"]) == {"phase_1", "phase_2"}


def test_device_deterministic(solver_mod):
    a = solver_mod.Solver(instance("mc_torus12x10")).solve(reoptLevel=0)
    b = solver_mod.Solver(instance("mc_torus12x10")).solve(reoptLevel=0)
    assert a["alm_inner"] == b["alm_inner"] and a["pobj"] == b["pobj"]


@pytest.mark.gpu
def test_coo_load_matches_file(solver_mod):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    a = solver_mod.Solver(instance("mc_torus12x10"))
    b = solver_mod.Solver(coo=inst.coo_arrays(inst.maxcut_torus_problem(12, 10, 5)))
    assert (a.m, a.dims, a.nslots, a.nnz) == (b.m, b.dims, b.nslots, b.nnz)
    ra, rb = a.solve(reoptLevel=0), b.solve(reoptLevel=0)
    assert ra["alm_inner"] == rb["alm_inner"] and ra["pobj"] == rb["pobj"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mc_rand200", "theta25x3"])
def test_stage_timing(solver_mod, name):
    sv = solver_mod.Solver(instance(name))
    r = sv.determine_rank()[0]
    out = sv.alm_throughput(0, 50, fixedRank=r, reoptLevel=0)
    assert out["done"] == 50
    ms = sv.time_stages(5)
    by = sv.stage_bytes()
    assert ms[0] > 0 and ms[2] > 0 and by[0] > 0 and by[2] > 0
    assert (ms[1] > 0) == (name.startswith("theta"))   # theta has the multi-slot trace constraint


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mc_rand200", "theta25x3", "rsparse60"])
def test_constraint_entry_auut_matches_pattern_path(solver_mod, name, monkeypatch):
    """k_auv_con (A(RR^T) straight from constraint entries) == SDDMM over the pattern + gather;
    k_auv_diag (MaxCut's identity-diagonal constraints: row-wise dot products, no index loads)
    the same values up to the compiler's FMA contraction of the lane sums (a few ulp)."""
    g = load_kernels(name)
    s = split_inputs(g)
    sv = solver_mod.Solver(instance(name))
    sv.set_rank([s["rank"]] * len(s["dims"]))
    sv.set_factor(solver_mod.R, s["R"])
    cvs, _, _ = sv.constr_rr()
    sv.time_auut(1)
    q = sv.get_vec(solver_mod.Q1)
    monkeypatch.setenv("LRS_NO_AUV_DIAG", "1")
    sv.time_auut(1)
    qc = sv.get_vec(solver_mod.Q1)
    if len(s["dims"]) == 1:
        assert np.array_equal(qc, cvs)          # same arithmetic, same order
        assert np.max(np.abs(q - cvs) / np.maximum(1.0, np.abs(cvs))) <= 1e-15
    assert rel_err(q, g["cvs_rr"]) < TOL
    assert sv.auut_bytes() > 0


_REGIME_SCRIPT = r"""
import importlib, json, sys
sys.path.insert(0, sys.argv[1])
s = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
out = {}
for name in sys.argv[2:]:
    if name.startswith("rsparse:"):   # in-memory random sparse SDP n:m (long rows: the wide path)
        n, m, r = map(int, name.split(":")[1:4])
        sv = s.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(n, m, 6, 7)))
        # a bounded ALM phase (150 inner iterations): the long-row kernels' arithmetic
        res = sv.solve(fixedRank=r, reoptLevel=0, skipADMM=1, almInnerBudget=150)
        out[name] = [res["alm_inner"], res["alm_pobj"], res["pobj"], res["admm_iter"]]
    else:
        sv = s.Solver(name)
        r = sv.solve(reoptLevel=0)
        out[name] = [r["alm_inner"], r["alm_pobj"], r["pobj"], r["admm_iter"]]
    sv.close()
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_bandwidth_regime_matches_latency_regime(tmp_path):
    """The large-n code paths (split stage A, unroll-1 B, occupancy grids) forced on small
    instances give the same solves as the latency-regime kernels (LRS_FORCE_REGIME)."""
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = [instance(n) for n in ("mc_torus12x10", "mc_rand300w", "theta25x3")] + ["rsparse:400:8000:16", "rsparse:4000:100000:128"]
    res = {}
    for reg in ("small", "large"):
        env = dict(os.environ, LRS_FORCE_REGIME=reg)
        p = subprocess.run([_sys.executable, "-c", _REGIME_SCRIPT, root] + names, env=env, capture_output=True,
                           text=True, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        res[reg] = json.loads(p.stdout.strip().splitlines()[-1])
    for nm in names:
        a, b = res["small"][nm], res["large"][nm]
        if "mc_" in nm:
            assert abs(a[0] - b[0]) <= 2, (nm, a, b)
            assert abs(a[1] - b[1]) <= 1e-8 * abs(a[1]), (nm, a, b)
        if "rsparse" in nm:
            assert a[0] == b[0] == 150, (nm, a, b)
            assert abs(a[1] - b[1]) <= 1e-8 * max(1.0, abs(a[1])), (nm, a, b)
        else:
            assert abs(a[2] - b[2]) <= 1e-6 * max(1.0, abs(a[2])), (nm, a, b)


# ranks across the register-blocking boundaries (NB = 1 / 2 / 4 tiles a side at r <= 16 /
# <= 192 / above) and the clamped column path (16 NB blocks wider than the row pitch: r = 17,
# 33 at ld = 24, 48)
GRAM_RANKS = [1, 5, 16, 17, 19, 33, 64, 128, 193, 200, 290, 512]


@pytest.mark.gpu
@pytest.mark.parametrize("r", GRAM_RANKS)
def test_gram_mfma_matches_fp64(solver_mod, r):
    """k_gram (v_mfma_f64_16x16x4_f64) == X^T X / ((U+V)/2)^T ((U+V)/2) in FP64
    (build_gram_from_factor / _from_average, lorads_logging.c:216-270)."""
    sv = solver_mod.Solver(instance("mc_rand300w"))
    _gram_check(solver_mod, sv, r)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [19, 64, 128, 290])
def test_gram_mfma_many_chunks(solver_mod, tmp_path, r):
    """The same at n = 4761 (64 row chunks, ragged last chunk)."""
    import importlib
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    path = str(tmp_path / "t.dat-s")
    inst.maxcut_torus(path, 69, 69, seed=3)
    sv = solver_mod.Solver(path)
    _gram_check(solver_mod, sv, r)


def _gram_check(solver_mod, sv, r):
    n = sv.dims[0]
    sv.set_rank([r])
    rng = np.random.default_rng(r)
    x, y = rng.standard_normal(n * r), rng.standard_normal(n * r)
    X, Y = x.reshape(r, n).T, y.reshape(r, n).T      # reference layout: column-major n x r
    sv.set_factor(solver_mod.R, x)
    g = sv.gram(0, solver_mod.R)
    ref = X.T @ X
    assert np.max(np.abs(g - ref)) <= 1e-12 * np.max(np.abs(ref))
    assert np.array_equal(g, g.T)
    sv.set_factor(solver_mod.U, x)
    sv.set_factor(solver_mod.V, y)
    g2 = sv.gram(0, solver_mod.U)
    A = 0.5 * (X + Y)
    ref2 = A.T @ A
    assert np.max(np.abs(g2 - ref2)) <= 1e-12 * np.max(np.abs(ref2))
    sv.close()


def _load_reopt():
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solves_reopt.json")) as f:
        return json.load(f)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(4))
def test_device_reopt_level1_matches_reference(solver_mod, case):
    """reoptLevel 1 (main.c:491-513, reopt() data/lorads_solver.c:1497-1539) against the
    reference's own reopt runs (tests/golden/solves_reopt.json, scripts/make_golden_reopt.py)."""
    g = _load_reopt()[case]
    r = g["result"]
    sv = solver_mod.Solver(instance(g["instance"]))
    res = sv.solve(reoptLevel=1)
    sv.close()
    sv0 = solver_mod.Solver(instance(g["instance"]))
    res0 = sv0.solve(reoptLevel=0)
    sv0.close()
    # main.c:493-495 on OUR level-0 result (theta / random-sparse trajectories differ from the
    # reference's in summation order, so whether a round is due is decided per run)
    t2 = 1e-5
    due = (res0["alm_gap"] > t2 or res0["alm_pinf"] > t2) and (res0["gap"] > t2 or res0["pinf"] > t2)
    if due:
        assert res["alm_outer"] > res0["alm_outer"]      # the reopt round's ALM ran
    else:
        assert res["alm_outer"] == res0["alm_outer"] and res["pobj"] == res0["pobj"]
    if r["alm_outer"] == g["level0_alm_outer"]:           # no round in the reference either
        assert abs(res["pobj"] - r["admm_pobj"]) <= 1e-6 * abs(r["admm_pobj"])
        return
    tol = 10 * (r["admm_gap"] + res["gap"]) + 2e-5
    assert abs(res["pobj"] - r["admm_pobj"]) <= tol * (1 + abs(r["admm_pobj"])), (res["pobj"], r["admm_pobj"], tol)
    if due:   # both ran the round: its ALM phase ends near the same point
        assert abs(res["alm_pobj"] - r["alm_pobj"]) <= tol * (1 + abs(r["alm_pobj"]))
    assert res["pinf"] <= 1e-4 and res["gap"] <= max(1e-4, 10 * r["admm_gap"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mc_torus12x10", "mc_rand200", "mc_rand300w", "rsparse60", "theta40"])
def test_latency_kernels_match_general(solver_mod, name, monkeypatch):
    """k_lat_a / k_lat_b (control wave + prefetching row waves) solve like the general row
    kernels k_it_a / k_it_b: same per-entry arithmetic, partial sums over other block
    partitions (MaxCut: inner iterations +-2, ALM objective 1e-8; all: final 1e-6)."""
    monkeypatch.setenv("LRS_SMALL", "0")   # path 0 = the latency kernels (not the single-workgroup loop)
    out = []
    for path in (0, 1):
        sv = solver_mod.Solver(instance(name))
        sv.set_kernel_path(path)
        r = sv.solve(reoptLevel=0)
        out.append((r, sv.kernel_path()))
        sv.close()
    (a, pa), (b, pb) = out
    assert pb == 1
    if name == "mc_torus12x10":   # sparse rows, 120 of them: every lane group resident, no teams
        assert pa == 0, "latency kernels not taken on a small sparse instance"
    if name.startswith("mc_"):
        assert abs(a["alm_inner"] - b["alm_inner"]) <= 2, (a["alm_inner"], b["alm_inner"])
        assert abs(a["alm_pobj"] - b["alm_pobj"]) <= 1e-8 * abs(b["alm_pobj"])
    tol = 1e-6 if name.startswith("mc_") else 10 * (a["gap"] + b["gap"]) + 1e-6
    assert abs(a["pobj"] - b["pobj"]) <= tol * max(1.0, abs(b["pobj"])), (a["pobj"], b["pobj"])


@pytest.mark.gpu
def test_latency_kernels_throughput_budget(solver_mod, monkeypatch):
    """The bench's fixed-budget ALM run (phase-1 exit off) does exactly `steps` iterations
    on the latency kernels, deterministically."""
    monkeypatch.setenv("LRS_SMALL", "0")
    sv = solver_mod.Solver(instance("mc_torus12x10"))
    r = sv.determine_rank()[0]
    outs = []
    for _ in range(2):
        o = sv.alm_throughput(0, 300, fixedRank=r, reoptLevel=0)
        outs.append(o["done"])
    assert sv.kernel_path() == 0
    assert outs == [300, 300]
    sv.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mc_torus12x10", "mc_rand200", "theta40", "theta25x3", "rsparse60"])
def test_dual_infeasibility_matches_dense_eig(solver_mod, name):
    """Dual infeasibility (calculate_dual_infeasibility_solver, data/lorads_solver.c:1396-1426)
    of the solve's multipliers: the device Lanczos' lambda_min(S_k), S = C - sum lambda_i A_i,
    against numpy's dense eigvalsh (1e-8 of ||S||), and the reference's ARPACK call
    (dsaupd "SA", ncv 40, tol 1e-2, data/lorads_sdp_conic.c:1636-1699) emulated with scipy's
    ARPACK within that tolerance; the l1 error as the reference forms it."""
    from golden_util import read_sdpa_dense
    import scipy.sparse.linalg as sla
    sv = solver_mod.Solver(instance(name))
    res = sv.solve(reoptLevel=0)
    lam = sv.get_vec(solver_mod.LAMBDA)
    l1, lmin = sv.dual_infeasibility()
    sv.close()
    m, dims, b, Cb, A = read_sdpa_dense(instance(name))
    err, cn1 = 0.0, sum(np.abs(Ck).sum() for Ck in Cb)
    for k, d in enumerate(dims):
        S = Cb[k].copy()
        for (i, blk), ents in A.items():
            if blk != k:
                continue
            for r, c, v in ents:
                S[r, c] -= lam[i] * v
                if r != c:
                    S[c, r] -= lam[i] * v
        ev = np.linalg.eigvalsh(S)[0]
        nS = max(1.0, np.abs(S).max() * d)
        # the reference's ARPACK stopping rule (tol 1e-2 relative Ritz estimate) or the device's
        # absolute one (1e-3 phase2Tol of the l_1 value): lrs_solver.cpp trl_min
        bar = 1e-2 * max(abs(ev), 1e-10) + 1e-3 * 1e-5 * (1 + cn1) + 1e-10 * nS
        assert ev <= lmin[k] + 1e-10 * nS and abs(lmin[k] - ev) <= bar, (k, lmin[k], ev)
        if d >= 40:
            w = sla.eigsh(S, k=1, which="SA", ncv=40, tol=1e-2, maxiter=600, return_eigenvectors=False)[0]
            assert abs(lmin[k] - w) <= bar + 1e-2 * abs(w), (k, lmin[k], w)
        err += abs(min(ev, 0.0))
    assert abs(l1 - err / (cn1 + 1)) <= 2e-2 * err / (cn1 + 1) + 1e-3 * 1e-5 * len(dims) + 1e-12
    # the solve evaluated it too (main.c:515) and reports l_inf = l_1 (1 + ||C||_1) / (1 + ||C||_inf)
    assert res["dinf"] >= 0
    assert abs(res["dinf"] - l1) <= 1e-8 * max(1.0, l1) + 1e-12


def test_more_than_256_cones_rejected(solver_mod, tmp_path):
    """The per-cone scalars live in fixed device slots (lrs_device.h TmpFinIdx, kMaxCones): at
    most 256 SDP cones, refused at load with a message instead of overrunning those slots."""
    def write(nb):
        lines = ["1", str(nb), " ".join(["2"] * nb), "1.0"]
        for k in range(1, nb + 1):
            lines += [f"0 {k} 1 1 1.0", f"1 {k} 1 1 1.0", f"1 {k} 2 2 1.0"]
        p = tmp_path / f"blocks{nb}.dat-s"
        p.write_text("\n".join(lines) + "\n")
        return str(p)
    sv = solver_mod.Solver(write(256))
    assert len(sv.dims) == 256
    sv.close()
    with pytest.raises(RuntimeError, match="256 SDP cones"):
        solver_mod.Solver(write(257))


def test_many_cones_stack_is_linear(solver_mod, tmp_path):
    """K = 100 independent copies of one small Lovasz-theta block (above the old 64-cone cap):
    the stacked SDP separates, so its optimum is K times the single block's (a size-independent
    property; both solved to the default tolerances)."""
    import importlib
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    rng = np.random.default_rng(5)
    n, ne, K = 10, 15, 100
    ei, ej = inst._random_edges(rng, n, ne)

    def write(nb):
        entries, b, con0 = [], [], 1
        for blk in range(1, nb + 1):
            entries += inst._theta_entries(n, ei, ej, blk, con0)
            b += [1.0] + [0.0] * ne
            con0 += 1 + ne
        p = str(tmp_path / f"theta_stack{nb}.dat-s")
        inst.write_sdpa(p, len(b), [n] * nb, np.array(b), entries)
        return p
    res = {}
    for nb in (1, K):
        sv = solver_mod.Solver(write(nb))
        res[nb] = sv.solve(reoptLevel=0)
        sv.close()
    one, many = res[1], res[K]
    assert abs(many["pobj"] - K * one["pobj"]) <= 1e-4 * abs(K * one["pobj"]), (many["pobj"], K * one["pobj"])
    assert abs(many["dobj"] - K * one["dobj"]) <= 1e-4 * abs(K * one["dobj"]), (many["dobj"], K * one["dobj"])


def test_dinf_step_cap_flagged(solver_mod, monkeypatch):
    """A dual-infeasibility eigen-solve that runs out of update iterations reports
    dinf_converged = 0 and the solve does not claim PRIMAL_DUAL_OPTIMAL on it (the Ritz value
    only bounds lambda_min from above).  LRS_TRL_NCV / LRS_TRL_MAXITER force a
    4-vector basis and no restart (the reference: ncv 40, 600 update iterations)."""
    monkeypatch.setenv("LRS_TRL_NCV", "4")
    monkeypatch.setenv("LRS_TRL_MAXITER", "0")
    sv = solver_mod.Solver(instance("theta40"))
    r = sv.solve(reoptLevel=0)
    sv.close()
    assert r["dinf_converged"] == 0 and r["dinf"] >= 0
    assert r["status"] != 1
    monkeypatch.delenv("LRS_TRL_NCV")
    monkeypatch.delenv("LRS_TRL_MAXITER")
    sv = solver_mod.Solver(instance("mc_rand200"))
    r = sv.solve(reoptLevel=0)
    sv.close()
    assert r["dinf_converged"] in (0, 1)


def test_time_limit_skips_dual_infeasibility(solver_mod):
    """main.c:450-454 / :505-510: a time-limit exit goes to END_SOLVING: no ADMM after the ALM
    phase, no dual infeasibility (dinf = -1, not evaluated), status TIME_LIMIT (4)."""
    sv = solver_mod.Solver(instance("theta40"))
    r = sv.solve(reoptLevel=1, timeSecLimit=1e-9)
    sv.close()
    assert r["status"] == 4 and r["dinf"] == -1.0 and r["dinf_converged"] == -1
    assert r["admm_iter"] == 0
