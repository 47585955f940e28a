"""The row partition of the sharded solve (lrs_shard_plan: shard_problem on the host, no
device) across processes: world_size 2 and 3 over gloo on CPU, each process computing its own
shard's plan from the same file and checking it against its peers' (all_gather_object):

  * the row blocks tile the cone, each owned range inside the shard's local rows;
  * halo plan: the rows shard p sends to q (global ids) are exactly q's halo rows from p;
  * every constraint is held by >= 1 shard and counted (primary) by exactly one;
  * the shared-constraint list is identical on every shard and is the set of constraints
    held by more than one.
SURVEY.md §8(e); DESIGN.md §6."""
import importlib
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "instances")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _check(plans, m_global):
    world = len(plans)
    n = plans[0]["n"]
    b = list(plans[0]["bounds"])
    assert b[0] == 0 and b[-1] == n and all(b[q] < b[q + 1] for q in range(world))
    for r, p in enumerate(plans):
        assert list(p["bounds"]) == b
        assert p["row0"] == b[r] and p["nown"] == b[r + 1] - b[r]
        lg = list(p["local_gid"])
        assert lg == sorted(lg) and set(range(b[r], b[r + 1])) <= set(lg)
    for p_ in range(world):
        for q in range(world):
            if p_ == q:
                continue
            sp = plans[p_]["send_ptr"]
            sent = list(plans[p_]["send_gid"][sp[q]:sp[q + 1]])
            halo_from_p = [g for g in plans[q]["local_gid"] if b[p_] <= g < b[p_ + 1]]
            assert sent == halo_from_p, (p_, q)
    held, prim = [0] * m_global, [0] * m_global
    for p in plans:
        for g, pr in zip(p["con_gid"], p["primary"]):
            held[g] += 1
            prim[g] += int(pr)
    assert all(h >= 1 for h in held) and all(c == 1 for c in prim)
    shared = [g for g in range(m_global) if held[g] > 1]
    for p in plans:
        assert list(p["shared_gid"]) == shared


def _worker(rank, world, port, names, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
        out = []
        for name in names:
            path = os.path.join(GOLD, f"{name}.dat-s")
            mine = solver.shard_plan(path, world, rank)
            allp = [None] * world
            dist.all_gather_object(allp, mine)
            with open(path) as f:
                lines = [ln for ln in f if ln.strip() and ln.lstrip()[0] not in '*"']
            _check(allp, int(lines[0].split()[0]))
            out.append((name, len(mine["shared_gid"])))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_plan_multiprocess(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    names = ["mc_torus12x10", "mc_rand200", "theta40", "rsparse60", "theta25x3"]
    procs = [ctx.Process(target=_worker, args=(r, world, port, names, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(world))
    shared = dict(res[0])
    assert shared["theta40"] > 0 and shared["rsparse60"] > 0   # constraints spanning row blocks


def test_shard_plan_single_process_bounds():
    sys.path.insert(0, ROOT)
    solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
    plans = [solver.shard_plan(os.path.join(GOLD, "mc_torus12x10.dat-s"), 4, r) for r in range(4)]
    _check(plans, 120)
    assert all(len(p["shared_gid"]) == 0 for p in plans)   # MaxCut: e_i e_i^T, never shared
