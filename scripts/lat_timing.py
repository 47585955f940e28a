#!/usr/bin/env python3
"""Diagnostics (GPU box): in-kernel phase stamps of the latency-regime kernels (k_lat_a /
k_lat_b) vs the general row kernels on the bench instance (timing build)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cols = int(sys.argv[2]) if len(sys.argv) > 2 else 100
timing = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "liblrsdp_timing.so") if not os.environ.get("LAT_PLAIN") else None
solver.load_library(timing)
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
path = bench.instance_for(0, rows, cols, cache)
for kp in (0, 1):
    sv = solver.Solver(path)
    sv.set_kernel_path(kp)
    r = sv.determine_rank()[0]
    kw = dict(fixedRank=r, reoptLevel=0)
    sv.alm_throughput(0, 300, **kw)
    out = sv.alm_throughput(0, 2000, **kw)
    stamps = [sv.debug_phase_times()]
    ms = sv.time_stages(200)
    stamps.append(sv.debug_phase_times())
    print(f"path={sv.kernel_path()} rank={r}: {out['done'] / out['seconds']:.1f} it/s; stage us {[round(x * 1e3, 2) for x in ms]}")
    for which, dbg in zip(("real loop", "time_stages"), stamps):
      if not dbg:
        continue
      ph, blk = dbg
      print(" --", which)
      for k, name in ((0, "A"), (2, "B")):
        t = ph[k]
        print(f"  K{name} stamps (us from entry):", [round((t[p] - t[0]) * 0.01, 2) if t[p] >= t[0] else None for p in range(12)])
        v = [(a, b) for a, b in blk[k] if a != 0 and b >= a]
        if v:
            f = min(a for a, _ in v); e = max(b for _, b in v)
            print(f"  K{name}: blocks {len(v)}, first entry -> last exit {(e - f) * 0.01:.2f} us, "
                  f"entry spread {(max(a for a, _ in v) - f) * 0.01:.2f} us, mean span {sum(b - a for a, b in v) / len(v) * 0.01:.2f} us")
    sv.close()

# per-block span by XCD (blockIdx % 8) of the last real-loop iteration
sv = solver.Solver(path)
r = sv.determine_rank()[0]
sv.alm_throughput(0, 300, fixedRank=r, reoptLevel=0)
dbg = sv.debug_phase_times()
if dbg:
    ph, blk = dbg
    for k, name in ((0, "A"), (2, "B")):
        v = [(q, a, b) for q, (a, b) in enumerate(blk[k]) if a != 0 and b >= a]
        if not v:
            continue
        f = min(a for _, a, _ in v)
        by = {}
        for q, a, b in v:
            by.setdefault(q % 8, []).append(((a - f) * 0.01, (b - f) * 0.01))
        print(f"K{name} per XCD: " + "  ".join(f"x{x}: exit mean {sum(e for _, e in l) / len(l):.2f} max {max(e for _, e in l):.2f}" for x, l in sorted(by.items())))
        worst = sorted(v, key=lambda t: -t[2])[:8]
        print(f"K{name} slowest blocks:", [(q, round((b - f) * 0.01, 2)) for q, a, b in worst])
sv.close()
