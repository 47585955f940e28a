#!/usr/bin/env python3
"""GPU box: phase times of the single-workgroup inner loop (kernel path 4) from the diagnostics
build's in-kernel stamps: theta3 at fixed rank 26, constant objective."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
solver.load_library(os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "liblrsdp_timing.so"))
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
name = sys.argv[1] if len(sys.argv) > 1 else "theta3"
sv = solver.Solver(inst.config_instance(name, cache))
sv.set_kernel_path(4)
sv.alm_throughput(0, 100, fixedRank=26, reoptLevel=0)
o = sv.alm_throughput(0, 2000, fixedRank=26, reoptLevel=0)
print(name, "%.1f us/it" % (o["seconds"] / max(1, o["done"]) * 1e6), "path", sv.kernel_path(), flush=True)
ph, blk = sv.debug_phase_times()
t = ph[3]
trips = max(1, int(t[15]))
names = ["control", "direction", "slots", "global+reduce", "line search", "R/S update", "rows", "global+reduce B"]
tot = sum(t[:8])
for q, nm in enumerate(names):
    print(f"  {nm:16s} {t[q] * 0.01 / trips:8.2f} us/trip ({100 * t[q] / max(1, tot):.0f} %)")
print(f"  wave 0: adjacency loops {t[8] * 0.01 / trips:.2f} us/trip, row epilogues {t[9] * 0.01 / trips:.2f} us/trip")
print(f"  trips {trips}, total {tot * 0.01 / trips:.2f} us/trip")
sv.close()
