"""The sharded solve's communication, recorded (include/lrsdp.h lrs_shard_comm_record / _log).

RCCL refuses two ranks on one GPU, so N > 1 RCCL runs happen only on a multi-GPU node.  What
can be checked here is the call sequence: both transports issue every halo exchange from one op
list (lrs_solver.cpp halo_ops: per peer, per cone, the send then the receive -- the body of the
RCCL transport's ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd), and record each all-reduce
where the RCCL transport calls ncclAllReduce.  On the loopback transport (world contexts on the
one GPU, the same kernels, plans and host control) every shard's log must then satisfy what RCCL
needs of the N processes:

  * every shard issues the same collectives (all-reduces of the same lengths) and the same
    halo groups in the same order (groups and collectives interleaved identically);
  * inside each group, the sends from p to q pair with q's receives from p: same count, same
    cone, same order;
  * a receive lands in the receiver's halo rows (past its owned rows), a send reads rows it owns.

Cases (verdict r5 item 5): theta40 (a shared trace constraint), rsparse60 (every constraint
shared) and the C5 structure at m = 10^5 (tiles, every row in every halo) over 2 / 3 / 4 shards,
three fused ALM trips each; and a whole mc_rand200 solve (ALM, ADMM with its CG dot-product
all-reduces, the dual infeasibility's Lanczos vector halos) over 2 and 3 shards.  The RCCL
transport with a one-rank communicator logs the same all-reduce sequence as a one-shard loopback."""
import importlib
import threading

import numpy as np
import pytest

from golden_util import instance

pytestmark = pytest.mark.gpu
GROUP, SEND, RECV, AR_DEV, AR_HOST = 0, 1, 2, 3, 4


@pytest.fixture(scope="module")
def mods():
    return (importlib.import_module("ltr-lowrank-sdp_amd.solver"),
            importlib.import_module("ltr-lowrank-sdp_amd.instances"))


def run_logged(solver, make, world, fn):
    grp = solver.LoopbackGroup(world)
    out, errs = [None] * world, []

    def work(r):
        try:
            sv = make()
            sv.shard_loopback(grp, r)
            sv.comm_record(True)
            res = fn(sv)
            out[r] = (sv.shard_info(), sv.comm_log(), res)
            sv.close()
        except Exception as e:   # reported below
            errs.append(f"rank {r}: {e!r}")

    ts = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(900)
    assert not any(t.is_alive() for t in ts), "sharded run did not finish"
    grp.close()
    assert not errs, errs
    return out


def skeleton(log):
    """The sequence of collectives and halo groups (p2p content collapsed): what every rank must
    issue identically."""
    return [tuple(x[[0, 2, 3]]) if x[0] in (AR_DEV, AR_HOST) else (GROUP, int(x[2])) for x in log
            if x[0] in (GROUP, AR_DEV, AR_HOST)]


def groups(log):
    """Per halo group, its ops (kind, peer, cone, count, offset)."""
    out, cur, left = [], None, 0
    for x in log:
        if x[0] == GROUP:
            cur, left = [], int(x[3])
            out.append(cur)
            if left == 0:
                cur = None
        elif x[0] in (SEND, RECV):
            assert cur is not None and left > 0, "p2p op outside a group"
            cur.append(tuple(int(v) for v in x))
            left -= 1
            if left == 0:
                cur = None
    assert cur is None, "unterminated group"
    return out


def check_logs(res, world):
    logs = [r[1] for r in res]
    assert all(len(lg) > 0 for lg in logs)
    sk = [skeleton(lg) for lg in logs]
    for r in range(1, world):
        assert sk[r] == sk[0], f"rank {r}: collectives / groups differ from rank 0"
    gs = [groups(lg) for lg in logs]
    ngroups = len(gs[0])
    assert all(len(g) == ngroups for g in gs)
    nsend = 0
    for gi in range(ngroups):
        for p in range(world):
            for q in range(world):
                if p == q:
                    continue
                sends = [(o[2], o[3]) for o in gs[p][gi] if o[0] == SEND and o[1] == q]
                recvs = [(o[2], o[3]) for o in gs[q][gi] if o[0] == RECV and o[1] == p]
                assert sends == recvs, (gi, p, q, sends, recvs)
                nsend += len(sends)
        for p in range(world):
            assert all(o[1] != p for o in gs[p][gi]), "a shard sends to itself"
    # receives land past the owned rows of a single-cone problem (halo rows); layouts of the
    # multi-cone ones are checked by the pairing above
    for (w, rk, row0, nown, nhalo), lg, _ in res:
        assert w == world and nhalo > 0
    return ngroups, nsend


@pytest.mark.parametrize("name,world", [("theta40", 2), ("theta40", 3), ("rsparse60", 2), ("rsparse60", 4)])
def test_trip_comm_pairs(mods, name, world):
    solver, _ = mods
    res = run_logged(solver, lambda: solver.Solver(instance(name)), world,
                     lambda sv: sv.alm_steps(3, reoptLevel=0))
    ng, ns = check_logs(res, world)
    assert ng >= 3 and ns > 0
    # per fused trip at least the direction halo and the stage totals' all-reduces
    n_ar = sum(1 for x in res[0][1] if x[0] == AR_DEV)
    assert n_ar >= 2 * 3


@pytest.mark.parametrize("world", [2, 4])
def test_trip_comm_pairs_c5_tiles(mods, world, monkeypatch):
    solver, inst = mods
    monkeypatch.setenv("LRS_SLOT_TILES", "1")
    coo = inst.coo_arrays(inst.random_sparse_problem(10000, 100000, 6, 5))
    res = run_logged(solver, lambda: solver.Solver(coo=coo), world,
                     lambda sv: sv.alm_steps(2, reoptLevel=0, fixedRank=128))
    check_logs(res, world)


@pytest.mark.parametrize("world", [2, 3])
def test_whole_solve_comm_pairs(mods, world):
    """ALM + ADMM (CG dot products, the solved factor's halo) + the dual infeasibility's Lanczos
    vector halos (halo groups of one cone's vector: cone >= 0 in the group record)."""
    solver, _ = mods
    res = run_logged(solver, lambda: solver.Solver(instance("mc_rand200")), world, lambda sv: sv.solve(reoptLevel=0))
    ng, _ = check_logs(res, world)
    lg = res[0][1]
    assert any(x[0] == GROUP and x[2] >= 0 for x in lg), "no vector halo (Lanczos) recorded"
    assert any(x[0] == AR_HOST for x in lg), "no host all-reduce (objective / Gram) recorded"
    objs = [r[2]["pobj"] for r in res]
    assert max(objs) == min(objs)   # every shard ends on the same summed values


def test_rccl_world1_logs_like_loopback(mods, monkeypatch):
    """A one-rank RCCL communicator (LRS_FORCE_SHARD=1 keeps the sharded iteration) records the
    same collectives as a one-shard loopback group on the same trips."""
    solver, _ = mods
    monkeypatch.setenv("LRS_FORCE_SHARD", "1")
    sv = solver.Solver(instance("theta40"))
    sv.shard_rccl(1, 0, solver.comm_unique_id())
    sv.comm_record(True)
    sv.alm_steps(3, reoptLevel=0)
    lr = sv.comm_log()
    sv.close()
    lb = run_logged(solver, lambda: solver.Solver(instance("theta40")), 1, lambda sv: sv.alm_steps(3, reoptLevel=0))
    assert skeleton(lr) == skeleton(lb[0][1])
    assert np.array_equal(lr[:, [0, 1, 2, 3]], lb[0][1][:, [0, 1, 2, 3]])
