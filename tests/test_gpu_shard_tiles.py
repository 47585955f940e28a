"""Sharded long-row iteration over the 2-D LDS tiles: each shard tiles
its owned rows only -- k_tile_a over the owned rows' lower slots, k_tile_b1 their S and
A(R_new R_new^T), k_slot_sv the S of the slots whose lower row is a halo row (the owned rows'
upper entries), k_tile_b2 the owned row tiles' S R_new -- and the stage totals meet in the
same all-reduces as the gather kernels' (lrs_kernels.hip enqueue_alm_stages).

Bars, as tests/test_gpu_shard.py and tests/test_gpu_c5_steps.py: the reference's own first K
trips (tau, ||G||^2, pinf) at 1e-9 relative on every shard, through the loopback transport
(world contexts on the one GPU, the kernels and plans the RCCL transport drives on N GPUs).
"""
import importlib
import os
import threading

import numpy as np
import pytest

from golden_util import GOLDEN, instance

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def mods():
    return (importlib.import_module("ltr-lowrank-sdp_amd.solver"),
            importlib.import_module("ltr-lowrank-sdp_amd.instances"))


def run_sharded(mod, make, world, fn, path=None):
    grp = mod.LoopbackGroup(world)
    out, errs = [None] * world, []

    def work(r):
        try:
            sv = make()
            sv.shard_loopback(grp, r)
            if path is not None:
                sv.set_kernel_path(path)
            res = fn(sv)
            out[r] = (sv.shard_info(), (sv.tile_info(), sv.tile_used()), res)
            sv.close()
        except Exception as e:   # reported below
            errs.append(f"rank {r}: {e!r}")

    ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    assert not any(t.is_alive() for t in ts), "sharded run did not finish"
    grp.close()
    assert not errs, errs
    return out


def check_trips(res, z, K):
    tau, rn, lag, pinf = z[f"K{K}_trips"][K - 1]
    for info, tiles, d in res:
        assert tiles[0][1] == 1 and tiles[1], ("shard without slot tiles", info, tiles)
        assert d["inner"] == K
        assert abs(d["tau"] - tau) <= TOL * abs(tau), (K, info, d["tau"], tau)
        assert abs(d["lag"] - lag) <= TOL * abs(lag), (K, info, d["lag"], lag)
        assert abs(d["pinf"] - pinf) <= TOL * max(abs(pinf), 1e-300), (K, info, d["pinf"], pinf)


@pytest.mark.parametrize("name,world", [("rsparse60", 2), ("rsparse60", 3), ("theta40", 3), ("mc_rand200", 2),
                                        ("theta25x3", 2)])
def test_sharded_slot_tiles_match_reference(mods, name, world, monkeypatch):
    """Small golden instances with the tiles forced (LRS_SLOT_TILES=1, kernel path 3):
    shared constraints (rsparse60, theta's trace), C in the slots, three cones."""
    solver, _ = mods
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    z = np.load(os.path.join(GOLDEN, f"steps_{name}.npz"))
    rank = int(z["rank_flag"])
    kw = {"reoptLevel": 0}
    if rank > 0:
        kw["fixedRank"] = rank
    for K in [int(k) for k in z["ks"]]:
        if z[f"K{K}_trips"].shape[0] < K:
            continue
        res = run_sharded(solver, lambda: solver.Solver(instance(name)), world, lambda sv: sv.alm_steps(K, **kw),
                          path=3)
        check_trips(res, z, K)


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_c5_tiles_match_reference(mods, world, monkeypatch):
    """BASELINE config C5's structure (n = 10^4, 6 entries per constraint, r = 128) at
    m = 10^5 (tests/golden/steps_c5_m1e5.npz, the reference's own trips) with the tiles
    forced, row-sharded 2 and 4 ways: every shard's halo is nearly every row, every
    constraint shared."""
    solver, inst = mods
    fx = os.path.join(GOLDEN, "steps_c5_m1e5.npz")
    z = np.load(fx)
    m = int(z["m"])
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    coo = inst.coo_arrays(inst.random_sparse_problem(10000, m, 6, 5))
    kw = {"reoptLevel": 0, "fixedRank": int(z["rank_flag"])}
    K = max(int(k) for k in z["ks"] if z[f"K{int(k)}_trips"].shape[0] >= int(k))
    K = min(K, 3)
    res = run_sharded(solver, lambda: solver.Solver(coo=coo), world, lambda sv: sv.alm_steps(K, **kw), path=3)
    check_trips(res, z, K)


def test_rccl_transport_tiles_world1(mods, monkeypatch):
    """The RCCL transport (a one-rank communicator; LRS_FORCE_SHARD=1 keeps the sharded
    iteration with its halo exchange and all-reduces) over the tiled long-row stages on the C5
    structure (m = 10^5, tiles forced): the reference's trips at 1e-9.  bench.py's `sharded` C5
    leg drives the same calls on N GPUs."""
    solver, inst = mods
    z = np.load(os.path.join(GOLDEN, "steps_c5_m1e5.npz"))
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    monkeypatch.setenv("LRS_FORCE_SHARD", "1")
    sv = solver.Solver(coo=inst.coo_arrays(inst.random_sparse_problem(10000, int(z["m"]), 6, 5)))
    sv.shard_rccl(1, 0, solver.comm_unique_id())
    sv.set_kernel_path(3)
    kw = {"reoptLevel": 0, "fixedRank": int(z["rank_flag"])}
    K = min(3, max(int(k) for k in z["ks"] if z[f"K{int(k)}_trips"].shape[0] >= int(k)))
    d = sv.alm_steps(K, **kw)
    res = [(sv.shard_info(), (sv.tile_info(), sv.tile_used()), d)]
    sv.close()
    check_trips(res, z, K)
