"""Multi-GPU replica bookkeeping for bench.py (SURVEY.md §8(e), round-1 scope).

One process per GPU, each solving its own instance (the reference's instance-level
batching, dataset/run_lorads.sh:85-114): no data-path collective.  The only
cross-rank traffic is the timing protocol: a barrier around the timed region and
one reduction of (iterations, seconds) -> (sum, max).  Works with any
torch.distributed backend ("nccl" = RCCL on the GPU box, "gloo" in the CPU tests).
"""
from __future__ import annotations


def barrier_sync(dist):
    """Barrier + device synchronisation on both sides (no-op without a process group)."""
    if dist is None:
        return
    import torch
    cuda = torch.cuda.is_available() and dist.get_backend() == "nccl"
    if cuda:
        torch.cuda.synchronize()
    dist.barrier()
    if cuda:
        torch.cuda.synchronize()


def aggregate(dist, done, seconds):
    """(iterations summed over ranks, seconds maxed over ranks)."""
    if dist is None:
        return float(done), float(seconds)
    import torch
    dev = "cuda" if (torch.cuda.is_available() and dist.get_backend() == "nccl") else "cpu"
    if dev == "cuda":
        dev = f"cuda:{torch.cuda.current_device()}"
    t = torch.tensor([float(done)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    s = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    return float(t.item()), float(s.item())
