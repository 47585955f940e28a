"""Sharded single-instance solve (include/lrsdp.h lrs_shard_*) on one
MI355X through the loopback transport: `world` contexts on the GPU, one host thread each,
collectives through host barriers + stream events.  The kernels, the row partition, the
halo plan and the host control are the ones the RCCL transport drives on N GPUs.

Bars: every shard runs the identical control (same iteration counts and objective bit
for bit); the sharded ALM phase reproduces the single-GPU one like the single-GPU one
reproduces the reference on MaxCut (inner iterations within +-2, objectives within 1e-6
relative: only the summation order differs)."""
import importlib
import threading

import pytest

from golden_util import instance

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver_mod():
    return importlib.import_module("ltr-lowrank-sdp_amd.solver")


def run_sharded(mod, path, world, fn):
    grp = mod.LoopbackGroup(world)
    out, errs = [None] * world, []

    def work(r):
        try:
            sv = mod.Solver(path)
            sv.shard_loopback(grp, r)
            out[r] = (sv.shard_info(), fn(sv))
            sv.close()
        except Exception as e:   # reported below
            errs.append(f"rank {r}: {e!r}")

    ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not any(t.is_alive() for t in ts), "sharded run did not finish"
    grp.close()
    assert not errs, errs
    return out


@pytest.mark.parametrize("name,world", [("mc_torus12x10", 2), ("mc_torus12x10", 4), ("mc_rand200", 3)])
def test_sharded_alm_phase_matches_single_gpu(solver_mod, name, world):
    kw = dict(reoptLevel=0, skipADMM=1)
    single = solver_mod.Solver(instance(name))
    n = single.dims[0]
    ref = single.solve(**kw)
    single.close()
    res = run_sharded(solver_mod, instance(name), world, lambda sv: sv.solve(**kw))
    infos = [r[0] for r in res]
    assert [i[1] for i in infos] == list(range(world))
    assert sum(i[3] for i in infos) == n                      # the row blocks cover the cone
    assert [i[2] for i in infos] == sorted(i[2] for i in infos)
    first = res[0][1]
    for _, r in res[1:]:
        for k in ("alm_inner", "alm_outer", "alm_pobj", "alm_dobj", "alm_pinf", "final_rank"):
            assert r[k] == first[k], (k, r[k], first[k])
    assert abs(first["alm_inner"] - ref["alm_inner"]) <= 2, (first["alm_inner"], ref["alm_inner"])
    assert first["final_rank"] == ref["final_rank"]
    for k in ("alm_pobj", "alm_dobj"):
        assert abs(first[k] - ref[k]) <= 1e-6 * max(1.0, abs(ref[k])), (k, first[k], ref[k])


def test_sharded_fixed_rank_throughput(solver_mod):
    """The bench's unit: a budget of inner iterations at fixed rank on every shard."""
    res = run_sharded(solver_mod, instance("mc_torus12x10"), 2,
                      lambda sv: sv.alm_throughput(0, 60, fixedRank=6, reoptLevel=0))
    assert all(r[1]["done"] == 60 for r in res)


def test_sharded_deterministic(solver_mod):
    kw = dict(reoptLevel=0, skipADMM=1)
    a = run_sharded(solver_mod, instance("mc_rand200"), 2, lambda sv: sv.solve(**kw))
    b = run_sharded(solver_mod, instance("mc_rand200"), 2, lambda sv: sv.solve(**kw))
    assert a[0][1]["alm_pobj"] == b[0][1]["alm_pobj"] and a[0][1]["alm_inner"] == b[0][1]["alm_inner"]


def test_rccl_transport_world1(solver_mod, monkeypatch):
    """The RCCL transport's plumbing on one GPU (a communicator of one rank: all-reduces,
    no halo peers; LRS_FORCE_SHARD=1, since one shard is otherwise the unsharded solve);
    bench.py drives the same calls on N GPUs under torch.distributed.run."""
    monkeypatch.setenv("LRS_FORCE_SHARD", "1")
    kw = dict(reoptLevel=0)
    single = solver_mod.Solver(instance("mc_torus12x10"))
    ref = single.solve(**kw)
    single.close()
    sv = solver_mod.Solver(instance("mc_torus12x10"))
    sv.shard_rccl(1, 0, solver_mod.comm_unique_id())
    assert sv.shard_info() == (1, 0, 0, 120, 0)
    assert sv.comm_ranks() == 1   # ncclCommCount of the communicator
    r = sv.solve(**kw)
    out = sv.alm_throughput(0, 40, fixedRank=6, reoptLevel=0)
    sv.close()
    assert abs(r["alm_inner"] - ref["alm_inner"]) <= 2
    assert abs(r["alm_pobj"] - ref["alm_pobj"]) <= 1e-6 * abs(ref["alm_pobj"])
    assert abs(r["pobj"] - ref["pobj"]) <= 1e-6 * abs(ref["pobj"])   # ADMM phase over RCCL too
    assert out["done"] == 40


def test_rccl_world1_is_unsharded(solver_mod):
    """lrs_shard_rccl(world = 1) leaves the context unsharded (no per-stage collectives)."""
    sv = solver_mod.Solver(instance("mc_torus12x10"))
    sv.shard_rccl(1, 0, solver_mod.comm_unique_id())
    assert sv.shard_info() == (1, 0, 0, 120, 0)
    r = sv.solve(reoptLevel=0)
    sv.close()
    assert r["dinf"] >= 0


@pytest.mark.parametrize("name,world", [("mc_torus12x10", 2), ("mc_torus12x10", 4), ("mc_rand200", 3),
                                        ("mc_rand300w", 2)])
def test_sharded_full_solve_matches_single_gpu(solver_mod, name, world):
    """ALM + ADMM sharded: the ADMM half-steps' CG runs on each shard's owned rows with its
    <p, Q>, <r, r> and ||b||_1 summed over the shards, the solved factor's
    halo rows exchanged after each half-step.  Every shard runs the identical control; the
    solve reproduces the single-GPU one (ALM inner iterations within +-2, ADMM iterations
    within +-1, objectives within 1e-6 relative)."""
    kw = dict(reoptLevel=0)
    single = solver_mod.Solver(instance(name))
    ref = single.solve(**kw)
    single.close()
    res = run_sharded(solver_mod, instance(name), world, lambda sv: sv.solve(**kw))
    first = res[0][1]
    for _, r in res[1:]:
        for k in ("alm_inner", "admm_iter", "cg_iter", "pobj", "dobj", "pinf", "gap", "final_rank"):
            assert r[k] == first[k], (k, r[k], first[k])
    assert abs(first["alm_inner"] - ref["alm_inner"]) <= 2, (first["alm_inner"], ref["alm_inner"])
    assert abs(first["admm_iter"] - ref["admm_iter"]) <= 1, (first["admm_iter"], ref["admm_iter"])
    for k in ("alm_pobj", "alm_dobj", "pobj", "dobj"):
        assert abs(first[k] - ref[k]) <= 1e-6 * max(1.0, abs(ref[k])), (k, first[k], ref[k])
    assert first["pinf"] <= max(1e-6, 10 * ref["pinf"])
    # the dual infeasibility is evaluated sharded too (trl_min over owned rows + halo)
    assert first["dinf"] >= 0 and first["dinf_converged"] == ref["dinf_converged"]
    assert first["status"] == ref["status"]


@pytest.mark.parametrize("name,world", [("theta40", 2), ("theta40", 3), ("rsparse60", 2), ("rsparse60", 4),
                                        ("mc_torus12x10", 3), ("theta25x3", 2), ("theta25x3", 3)])
def test_sharded_steps_match_reference(solver_mod, name, world):
    """Constraints spanning row blocks (theta's trace and cross-block edges, rsparse's random
    multi-entry rows; theta25x3: three cones, each split across the shards): every holder sums
    its owned-slot entries, the shared constraints'
    sums meet in an all-reduce, and the primary holder alone counts them in the line-search
    dots and residuals.  K fused ALM trips on every shard against the reference's own K trips
    (tests/golden/steps_<name>.npz): tau, ||G||^2 and pinf to 1e-9 relative."""
    import os
    import numpy as np
    from golden_util import GOLDEN
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    for K in [int(k) for k in z["ks"]]:
        trips = z[f"K{K}_trips"]
        if trips.shape[0] < K:
            continue
        res = run_sharded(solver_mod, instance(name), world, lambda sv: sv.alm_steps(K, **kw))
        tau, rn, lag, pinf = trips[K - 1]
        for info, d in res:
            assert d["inner"] == K
            assert abs(d["tau"] - tau) <= 1e-9 * abs(tau), (K, d["tau"], tau)
            assert abs(d["lag"] - lag) <= 1e-9 * abs(lag), (K, d["lag"], lag)
            assert abs(d["pinf"] - pinf) <= 1e-9 * max(abs(pinf), 1e-300), (K, d["pinf"], pinf)


@pytest.mark.parametrize("name,world", [("theta40", 2), ("rsparse60", 3), ("theta25x3", 2)])
def test_sharded_full_solve_shared_constraints(solver_mod, name, world):
    """Whole ALM + ADMM solves with shared constraints (the CG direction's halo rows exchanged
    before every matvec, A(.) of shared constraints summed over the holders): every shard
    identical; against the single-GPU solve within the bar of the theta / random-sparse golden
    solves (thousands of L-BFGS steps, FP64 summation order differs): objectives within
    10 x the certified gaps, pinf <= 1e-4, the same final rank."""
    kw = dict(reoptLevel=0)
    single = solver_mod.Solver(instance(name))
    ref = single.solve(**kw)
    single.close()
    res = run_sharded(solver_mod, instance(name), world, lambda sv: sv.solve(**kw))
    first = res[0][1]
    for _, r in res[1:]:
        for k in ("alm_inner", "admm_iter", "pobj", "dobj", "pinf", "gap", "final_rank"):
            assert r[k] == first[k], (k, r[k], first[k])
    tol = 10 * (ref["gap"] + first["gap"]) + 1e-6
    for k in ("pobj", "dobj"):
        assert abs(first[k] - ref[k]) <= tol * (1 + abs(ref[k])), (k, first[k], ref[k], tol)
    assert first["pinf"] <= 1e-4
    assert first["final_rank"] == ref["final_rank"]
