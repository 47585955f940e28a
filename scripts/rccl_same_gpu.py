#!/usr/bin/env python3
"""Probe (GPU box): can two RCCL ranks share one GPU?  Prints the all-reduce result or the error."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world)
        x = torch.full((4,), float(rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        print(f"rank {rank}: {x.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:   # report, do not hang
        print(f"rank {rank}: error {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=work, args=(r, 2, 29517)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(90)
        if p.exitcode is None:
            p.kill()
    print("exit codes", [p.exitcode for p in ps], flush=True)
