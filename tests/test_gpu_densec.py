"""Dense objective on the FP64 matrix cores (BASELINE config C5b):
C kept as a full n x n matrix out of the slot pattern; every C-term of the iteration is a
product with it (k_cgemm: C D with <R, C D>, <D, C D> for the line search, C R carried through
stage B, C Y in the ADMM right-hand side, C q_j in the dual-infeasibility Lanczos).  The
reference's own dense branches (fds_syr2k in LORADSUVt lorads_alg_common.c:72-89,
dataMatDenseMultiRkMat lorads_sdp_data.c:948-973) are the oracle:

* steps_rdense300.npz (scripts/make_golden_steps.py): K = 1..5 trips of the reference's inner
  loop on a C5b-structured instance (n = 300, m = 3000, dense random C) -- tau, R_K, G_K,
  A(R_K R_K^T), the L-BFGS pair to 1e-9 (the bar of test_gpu_steps), through the dense path
  (LRS_DENSE_C=1) on kernel paths 1, 2 and 3 (the long-row kernels k_wide_a / k_wide_b, which
  C5b's ~1 200-entry rows take) and through the slot path (LRS_DENSE_C=0);
* the theta fixtures (C = -J, dense) through the dense path, same bar;
* solves_densec.json (scripts/make_golden_densec.py): whole reference solves; the ALM objectives
  within 1e-4 relative (the reference's own ALM primal-dual gap on them is 1.4e-5 / 2.3e-5 and the
  40 000-trip trajectories are chaotic), the final objectives within 1e-4;
* dense and slot paths on theta40: the same optimum (ALM objectives 1e-4; final objectives
  within twice the reference's certified bracket width; dual infeasibility within 5 %).
"""
import hashlib
import importlib
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, instance, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


@pytest.fixture(scope="module")
def gen_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("densec")


def _rdense(gen_dir, n, m, k, seed, sha=None):
    inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
    path = str(gen_dir / f"rdense_{n}_{m}_{k}_{seed}.dat-s")
    if not os.path.exists(path):
        inst.random_sparse(path, n, m, k, seed, dense_c=True)
    if sha is not None:
        assert hashlib.sha256(open(path, "rb").read()).hexdigest() == sha, "generator drifted"
    return path


class dense_mode:
    """LRS_DENSE_C for the problems loaded inside the block (read at load time)."""

    def __init__(self, v):
        self.v = v

    def __enter__(self):
        self.old = os.environ.get("LRS_DENSE_C")
        os.environ["LRS_DENSE_C"] = self.v

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop("LRS_DENSE_C", None)
        else:
            os.environ["LRS_DENSE_C"] = self.old


def _steps_check(solver_mod, path, z, mode, kpath):
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    with dense_mode(mode):
        sv = solver_mod.Solver(path)
    sv.set_kernel_path(kpath)
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
        for key in ("R", "G", "cvs", "s", "y"):
            e = rel_err(d[key], z[f"K{K}_{key}"])
            assert e < TOL, (K, key, e)
        assert sv.kernel_path() == (1 if kpath else sv.kernel_path())   # path 0: latency kernels when they fit
    sv.close()


@pytest.mark.parametrize("mode,kpath", [("1", 0), ("1", 1), ("1", 2), ("1", 3), ("0", 1)])
def test_dense_objective_steps_match_reference(solver_mod, gen_dir, mode, kpath):
    z = np.load(os.path.join(GOLDEN, "steps_rdense300.npz"))
    _steps_check(solver_mod, _rdense(gen_dir, 300, 3000, 6, 7), z, mode, kpath)


@pytest.mark.parametrize("const", ["0", "1"])
@pytest.mark.parametrize("name,kpath", [("theta40", 0), ("theta40", 1), ("theta40", 2), ("theta25x3", 0),
                                        ("theta25x3", 1), ("theta25x3", 2)])
def test_theta_dense_objective_steps_match_reference(solver_mod, name, kpath, const, monkeypatch):
    """theta's C = -J through the dense path: as a full matrix on the matrix cores (k_cgemm,
    LRS_CONST_C=0) and as the constant objective's rank-one products (k_cjx, the default for a
    block whose C entries are all equal)."""
    monkeypatch.setenv("LRS_CONST_C", const)
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    _steps_check(solver_mod, instance(name), z, "1", kpath)


def _solves():
    with open(os.path.join(GOLDEN, "solves_densec.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("idx", [0, 1])
def test_dense_objective_solve_matches_reference(solver_mod, gen_dir, idx):
    g = _solves()[idx]
    path = _rdense(gen_dir, g["n"], g["m"], g["k"], g["seed"], g["sha256"])
    kw = {}
    for k, v in zip(g["flags"][0::2], g["flags"][1::2]):
        k = k.lstrip("-")
        kw[k] = int(v) if k in ("reoptLevel", "fixedRank") else float(v)
    with dense_mode("1"):
        sv = solver_mod.Solver(path)
    res = sv.solve(**kw)
    sv.close()
    ref = g["result"]
    for ours, theirs in (("alm_pobj", "alm_pobj"), ("alm_dobj", "alm_dobj")):
        assert abs(res[ours] - ref[theirs]) <= 1e-4 * abs(ref[theirs]), (ours, res[ours], ref[theirs])
    j = g["json"]["metrics"]
    assert abs(res["pobj"] - j["primal_obj"]) <= 1e-4 * abs(j["primal_obj"]), (res["pobj"], j["primal_obj"])
    assert abs(res["dobj"] - j["dual_obj"]) <= 1e-4 * abs(j["dual_obj"]), (res["dobj"], j["dual_obj"])


@pytest.mark.parametrize("const", ["0", "1"])
def test_dense_and_slot_paths_agree_on_theta(solver_mod, const, monkeypatch):
    monkeypatch.setenv("LRS_CONST_C", const)
    out = {}
    for mode in ("0", "1"):
        with dense_mode(mode):
            sv = solver_mod.Solver(instance("theta40"))
        out[mode] = sv.solve(reoptLevel=0)
        sv.close()
    a, b = out["0"], out["1"]
    print({k: (a[k], b[k]) for k in ("alm_inner", "alm_pobj", "alm_dobj", "pobj", "dobj", "dinf", "admm_iter")})
    # the two paths round differently, so their ~1 000-trip ALM trajectories part: the ALM
    # objectives agree to the phase-1 tolerance, the final (ADMM) ones and the dual
    # infeasibility to the solve's
    for key in ("alm_pobj", "alm_dobj"):
        assert abs(a[key] - b[key]) <= 1e-4 * max(1.0, abs(a[key])), (key, a[key], b[key])
    # final objectives: within twice the width of the reference's own certified bracket
    # |primal_obj - dual_obj| on this instance (tests/golden/solves.json, 1.36e-3)
    j = [g for g in json.load(open(os.path.join(GOLDEN, "solves.json"))) if g["instance"] == "theta40"][0]
    width = abs(j["json"]["metrics"]["primal_obj"] - j["json"]["metrics"]["dual_obj"])
    for key in ("pobj", "dobj"):
        assert abs(a[key] - b[key]) <= 2 * width, (key, a[key], b[key], width)
    assert abs(a["dinf"] - b["dinf"]) <= 0.05 * abs(a["dinf"]), (a["dinf"], b["dinf"])


@pytest.mark.parametrize("kpath,tiles", [(0, "0"), (3, "0"), (3, "1"), (3, "2d")])
def test_dense_and_slot_paths_agree_per_trip_at_n2000(solver_mod, gen_dir, kpath, tiles, monkeypatch):
    """Past the fixtures' size (n = 2000, m = 100 000, r = 64; the reference's dense branches
    take minutes per trip here): the dense path and the slot path -- two independent
    evaluations of the same iteration -- give the same K = 1..3 trips (tau to 1e-9, R_K, G_K
    to 1e-9)."""
    path = _rdense(gen_dir, 2000, 100000, 6, 5)
    # tiles "1": the column-tiled long-row kernels (LRS_TILES, experimental, read at the
    # workspace allocation and the first enqueue of the process)
    # tiles "2d": the 2-D LDS tiles of the long-row stages and of A(X Y^T) (DESIGN.md §4.5,
    # read when the problem is loaded), on both the dense and the slot path
    monkeypatch.setenv("LRS_TILES", "0" if tiles == "2d" else tiles)
    if tiles == "2d":
        monkeypatch.setenv("LRS_SLOT_TILES", "1")
        monkeypatch.setenv("LRS_AUV_TILES", "1")
    out = {}
    for mode in ("0", "1"):
        with dense_mode(mode):
            sv = solver_mod.Solver(path)
        sv.set_kernel_path(kpath)   # 3: the long-row kernels, C5b's path at full size
        out[mode] = [sv.alm_steps(K, reoptLevel=0, fixedRank=64) for K in (1, 2, 3)]
        sv.close()
    for a, b in zip(out["0"], out["1"]):
        assert abs(a["tau"] - b["tau"]) <= TOL * abs(a["tau"]), (a["tau"], b["tau"])
        for key in ("R", "G", "cvs"):
            # with the 2-D tiles both paths' A(R R^T) sums each dot over r in sequence: the
            # constraint values here are ~1e-11 cancellations of O(1) products, so they carry
            # the iterate's 1e-16 differences amplified to ~1e-9 (R and G stay at 1e-9)
            tol = 1e-8 if (tiles == "2d" and key == "cvs") else TOL
            assert rel_err(a[key], b[key]) < tol, (key, rel_err(a[key], b[key]))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dense_objective_steps_match_reference(solver_mod, gen_dir, world):
    """A dense objective sharded by rows (lrs_problem.cpp shard_problem): each shard holds C's
    owned row block (owned rows x all n columns) and every row in its halo, so C_own D / C_own R
    (k_cgemm over the row block) read a complete factor after the halo exchange, and <R, C D>,
    <D, C D> are owned-row partials summed with the stage totals.  K trips on every shard
    against the reference's own (steps_rdense300): tau, ||G||^2 and pinf to 1e-9."""
    from test_gpu_shard import run_sharded
    z = np.load(os.path.join(GOLDEN, "steps_rdense300.npz"))
    path = _rdense(gen_dir, 300, 3000, 6, 7)
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    with dense_mode("1"):
        for K in [int(k) for k in z["ks"]]:
            trips = z[f"K{K}_trips"]
            if trips.shape[0] < K:
                continue
            res = run_sharded(solver_mod, path, world, lambda sv: sv.alm_steps(K, **kw))
            tau, rn, lag, pinf = trips[K - 1]
            for info, d in res:
                assert info[0] == world and info[4] > 0   # sharded, with a halo
                assert d["inner"] == K
                assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, d["tau"], tau)
                assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, d["lag"], lag)
                assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)


def test_sharded_dense_objective_solve_matches_single_gpu(solver_mod, gen_dir):
    """Whole sharded ALM + ADMM solve with the dense objective (C_own Y in the ADMM right-hand
    side, C_own q in the dual-infeasibility Lanczos) against the single-GPU solve: every shard
    identical; objectives within 10 x the certified gaps, the same final rank and status."""
    from test_gpu_shard import run_sharded
    g = _solves()[0]
    path = _rdense(gen_dir, g["n"], g["m"], g["k"], g["seed"], g["sha256"])
    kw = dict(reoptLevel=0)
    with dense_mode("1"):
        single = solver_mod.Solver(path)
        ref = single.solve(**kw)
        single.close()
        res = run_sharded(solver_mod, path, 2, lambda sv: sv.solve(**kw))
    first = res[0][1]
    for _, r in res[1:]:
        for k in ("alm_inner", "admm_iter", "pobj", "dobj", "pinf", "gap", "final_rank", "status"):
            assert r[k] == first[k], (k, r[k], first[k])
    tol = 10 * (ref["gap"] + first["gap"]) + 1e-6
    for k in ("pobj", "dobj"):
        assert abs(first[k] - ref[k]) <= tol * (1 + abs(ref[k])), (k, first[k], ref[k], tol)
    assert first["final_rank"] == ref["final_rank"] and first["status"] == ref["status"]
    assert first["dinf"] >= 0


@pytest.mark.parametrize("split", ["1", "3", "auto"])
def test_split_k_cgemm_per_trip_at_n2500(solver_mod, gen_dir, split, monkeypatch):
    """k_cgemm2 (dense cones of >= 2048 rows: full-width 32 x 128 output tiles, split over K
    into slabs that k_cgemm2_fin adds in slab order) against the slot path, K = 1..3 trips at
    n = 2500, r = 96 (tau, R_K, G_K to 1e-9): S = 1 (fused epilogue), S = 3 and the size rule;
    the ADMM / objective products through the same kernels (final objectives within 1e-6)."""
    path = _rdense(gen_dir, 2500, 60000, 6, 11)
    if split != "auto":
        monkeypatch.setenv("LRS_CG_SPLIT", split)
    out = {}
    for mode in ("0", "1"):
        with dense_mode(mode):
            sv = solver_mod.Solver(path)
        out[mode] = [sv.alm_steps(K, reoptLevel=0, fixedRank=96) for K in (1, 2, 3)]
        sv.close()
    for a, b in zip(out["0"], out["1"]):
        assert abs(a["tau"] - b["tau"]) <= TOL * abs(a["tau"]), (a["tau"], b["tau"])
        for key in ("R", "G"):
            assert rel_err(a[key], b[key]) < TOL, (key, rel_err(a[key], b[key]))
