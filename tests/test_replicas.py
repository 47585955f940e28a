"""Multi-process (world_size 2, gloo on CPU) coverage of bench.py's N>1 path:
per-rank instances, barrier and the (sum, max) timing reduction (ltr-lowrank-sdp_amd/replicas.py)."""
import importlib
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, tmpdir, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        replicas = importlib.import_module("ltr-lowrank-sdp_amd.replicas")
        bench = importlib.import_module("bench")
        path = bench.instance_for(rank, 6, 7, tmpdir)
        replicas.barrier_sync(dist)
        done, secs = replicas.aggregate(dist, 100 + rank, 1.5 + rank)
        q.put((rank, path, done, secs))
    finally:
        dist.destroy_process_group()


def test_replicas_world2(tmp_path):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    (r0, p0, d0, s0), (r1, p1, d1, s1) = res
    assert (d0, s0) == (201.0, 2.5) and (d1, s1) == (201.0, 2.5)
    # one distinct instance per rank (weak scaling: per-GPU work fixed)
    assert p0 != p1 and os.path.exists(p0) and os.path.exists(p1)
    assert open(p0).read() != open(p1).read()


def test_aggregate_single_process():
    sys.path.insert(0, ROOT)
    replicas = importlib.import_module("ltr-lowrank-sdp_amd.replicas")
    assert replicas.aggregate(None, 7, 0.25) == (7.0, 0.25)
    replicas.barrier_sync(None)
