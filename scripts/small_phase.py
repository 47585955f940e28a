#!/usr/bin/env python3
"""Diagnostics (GPU box): where the single-workgroup inner loop (k_small_alm)
spends a trip, from the in-kernel phase ticks of the diagnostics build (liblrsdp_timing.so,
g_phase[3]: thread 0's wall clock at 100 MHz between the loop's barriers), on one theta solve."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
inst = importlib.import_module("ltr-lowrank-sdp_amd.instances")
timing = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "liblrsdp_timing.so")
solver.load_library(timing)
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
sdplib = {"reoptLevel": 0, "heuristicFactor": 1.0, "phase1Tol": 1e-3, "rhoMax": 5000.0}
NAMES = ["control", "direction", "slots", "global+reduce", "linesearch", "R/S update", "rows", "constraints+reduce",
         "rows:adjacency", "rows:epilogue"]
for name in sys.argv[1:] or ["theta3"]:
    os.environ["LRS_SMALL"] = "1"
    sv = solver.Solver(inst.config_instance(name, cache))
    before = sv.debug_phase_times()[0]
    t0 = time.perf_counter()
    r = sv.solve(**sdplib)
    wall = time.perf_counter() - t0
    after = sv.debug_phase_times()[0]
    ph = [a - b for a, b in zip(after[3], before[3])]
    cg = [a - b for a, b in zip(after[1], before[1])]
    trips = max(1, ph[15])
    print(f"{name}: solve {wall:.3f} s alm {r['alm_time']:.3f} s ({r['alm_inner']} inner) admm {r['admm_time']:.3f} s "
          f"({r['admm_iter']} it, cg {r['cg_iter']}); k_small_alm trips {ph[15]}")
    tot = sum(ph[q] for q in range(8))
    print("  us/trip:", " ".join(f"{NAMES[q]} {ph[q] * 0.01 / trips:.2f}" for q in range(10)),
          f"| sum {tot * 0.01 / trips:.2f}")
    if cg[15]:
        nl = cg[15]
        print(f"  k_small_cg launches {nl}, CG iterations {cg[14]} ({cg[14] / nl:.2f} a launch); us/launch:",
              " ".join(f"{k} {cg[q] * 0.01 / nl:.2f}" for q, k in zip(range(8, 13), ["staging", "rhs", "first-residual",
                                                                               "cg-iterations", "refresh"])),
              f"| per CG iteration {cg[11] * 0.01 / max(1, cg[14]):.2f}")
        print("  first residual's operator passes (us/launch):",
              " ".join(f"{k} {cg[q] * 0.01 / nl:.2f}" for q, k in zip(range(4, 8), ["prod", "constraints", "slots", "apply"])))
    sv.close()
