#!/usr/bin/env python3
"""GPU box: the north-star workload (G81-structured torus 100 x 200, r = 64) on each kernel path
(lrs_set_kernel_path: 0 auto, 2 bandwidth regime split, 3 + the long-row neighbour kernels
k_wide_a / k_wide_b on every row) and with the environment's switches, interleaved rounds:
ALM it/s over 2 000 trips and lrs_time_stages per stage.  argv: rounds (default 2)."""
import importlib
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
td = tempfile.mkdtemp()
path = os.path.join(td, "g81.dat-s")
inst.maxcut_torus(path, 100, 200, seed=81)
kw = dict(fixedRank=64, reoptLevel=0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for rnd in range(rounds):
    for kp in (0, 2, 3):
        sv = solver.Solver(path)
        sv.set_kernel_path(kp)
        sv.alm_throughput(0, 100, **kw)
        o = sv.alm_throughput(0, 2000, **kw)
        ms = sv.time_stages(100)
        print(f"round {rnd} path {kp} (ran {sv.kernel_path()}): {o['done'] / o['seconds']:.0f} it/s; stages us "
              f"{[round(x * 1e3, 2) for x in ms]}", flush=True)
        sv.close()
