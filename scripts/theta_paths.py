#!/usr/bin/env python3
"""GPU box: theta-class fixed-rank ALM us/iteration under a forced kernel path (argv: name, path,
iterations); LRS_CONST_C / LRS_SMALL in the environment pick the objective form and the
single-workgroup loop (read at upload)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
name = sys.argv[1] if len(sys.argv) > 1 else "theta3x3"
path = int(sys.argv[2]) if len(sys.argv) > 2 else 0
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
sv = solver.Solver(inst.config_instance(name, cache))
sv.set_kernel_path(path)
sv.alm_throughput(0, 200, fixedRank=26, reoptLevel=0)
o = sv.alm_throughput(0, iters, fixedRank=26, reoptLevel=0)
ms = sv.time_stages(100)
print(f"{name} const_c={os.environ.get('LRS_CONST_C', '-')} small={os.environ.get('LRS_SMALL', '-')} path={path} "
      f"ran={sv.kernel_path()}: {o['seconds'] / max(1, o['done']) * 1e6:.1f} us/it; stages us "
      f"{[round(x * 1e3, 2) for x in ms]}", flush=True)
sv.close()
