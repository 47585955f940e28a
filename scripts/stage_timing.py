#!/usr/bin/env python3
"""Diagnostics (GPU box): where the split ALM iteration spends its time on the bench
instance.  Prints graph vs eager throughput, per-stage HIP-event durations and the
in-kernel phase timestamps of the diagnostics build (liblrsdp_timing.so)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT))
solver = importlib.import_module("ltr-lowrank-sdp_amd.solver")
bench = importlib.import_module("bench")

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100
cols = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
timing = os.path.join(ROOT, "ltr-lowrank-sdp_amd", "_build", "liblrsdp_timing.so")
solver.load_library(timing if os.path.exists(timing) else None)
cache = os.path.join(ROOT, ".bench_instances")
os.makedirs(cache, exist_ok=True)
path = bench.instance_for(0, rows, cols, cache)
for ng in ("1", "0"):
    os.environ["LRS_GRAPHS"] = "0" if ng == "1" else "1"
    sv = solver.Solver(path)
    r = rank or sv.determine_rank()[0]
    kw = dict(fixedRank=r, reoptLevel=0)
    sv.alm_throughput(0, 300, **kw)
    out = sv.alm_throughput(0, 2000, **kw)
    print(f"graphs={'off' if ng == '1' else 'on'} rank={r}: {out['done'] / out['seconds']:.1f} it/s "
          f"({out['seconds'] * 1e6 / out['done']:.1f} us/it)")
    for mode in (("throughput", "profile") if ng == "1" else ()):
        if mode == "profile":
            ms, done = sv.profile_stages(600, **kw)
            print("stage us (events):", [round(x * 1e3, 2) for x in ms], "sum", round(sum(ms) * 1e3, 2),
                  "iters", done)
        print(f"-- in-kernel stamps of the last iteration ({mode} run)")
        dbg = sv.debug_phase_times()
        if dbg:
            ph, blk = dbg
            names = [["entry", "ctrl-load", "reduce10", "ctrl+glob", "start", "rows", "partials"],
                     ["entry", "pinf", "gather_q", "partials"],
                     ["entry", "reduce", "linesearch", "rows", "partials"]]
            for k in range(3):
                t = ph[k]
                seq = [f"{names[k][p]}:{(t[p] - t[p - 1]) * 0.01:.2f}" for p in range(1, len(names[k]))]
                print(f"K{'AGB'[k]} phases (us):", " ".join(seq))
            # latency kernels (k_lat_a / k_lat_b, block 0): row waves' own operands / neighbours
            # loaded, the control wave's partial sums and control step, from the block's entry
            a0, b0 = ph[0], ph[2]
            if a0[0] and a0[7] and a0[8]:
                print("k_lat_a block 0 (us from entry): own rows", round((a0[1] - a0[0]) * 0.01, 2), "neighbours",
                      round((a0[2] - a0[0]) * 0.01, 2), "| ctrl partials summed", round((a0[8] - a0[0]) * 0.01, 2),
                      "ctrl_step done", round((a0[7] - a0[0]) * 0.01, 2), "| barrier", round((a0[3] - a0[0]) * 0.01, 2),
                      "rows done", round((a0[5] - a0[0]) * 0.01, 2), "partials stored", round((a0[6] - a0[0]) * 0.01, 2),
                      "| row header", round((a0[10] - a0[0]) * 0.01, 2), "control words", round((a0[9] - a0[0]) * 0.01, 2),
                      "ctrl wave's control block", round((a0[11] - a0[0]) * 0.01, 2))
            if b0[0] and b0[7] and b0[8]:
                print("k_lat_b block 0 (us from entry): own rows", round((b0[5] - b0[0]) * 0.01, 2), "neighbours",
                      round((b0[6] - b0[0]) * 0.01, 2), "| ctrl partials summed", round((b0[8] - b0[0]) * 0.01, 2),
                      "line search done", round((b0[7] - b0[0]) * 0.01, 2), "| barrier", round((b0[2] - b0[0]) * 0.01, 2),
                      "rows done", round((b0[3] - b0[0]) * 0.01, 2), "partials stored", round((b0[4] - b0[0]) * 0.01, 2))
            t = ph[2]
            if t[6] and t[11]:
                print("KB rows detail (us from LS end): header", round((t[6] - t[2]) * 0.01, 2), "chunk1 data",
                      round((t[7] - t[2]) * 0.01, 2), "chunk1 done", round((t[8] - t[2]) * 0.01, 2), "chunk2 data",
                      round((t[9] - t[2]) * 0.01, 2), "chunk2 done", round((t[10] - t[2]) * 0.01, 2), "epilogue",
                      round((t[11] - t[2]) * 0.01, 2), "rows end", round((t[3] - t[2]) * 0.01, 2))
            # per-block spans of the last full iteration (valid blocks: entry != 0)
            spans = []
            ks = [k for k in range(3) if any(a != 0 for a, _ in blk[k])]
            for k in ks:
                v = [(a, b) for a, b in blk[k] if a != 0 and b >= a]
                spans.append((min(a for a, _ in v), max(a for a, _ in v), max(b for _, b in v), len(v),
                              sum(b - a for a, b in v) / len(v)))
            for q, k in enumerate(ks):
                f, l, e, nb, av = spans[q]
                line = (f"K{'AGB'[k]}: blocks {nb} first-entry->last-entry {(l - f) * 0.01:.2f} us, "
                        f"first-entry->last-exit {(e - f) * 0.01:.2f} us, mean block span {av * 0.01:.2f} us")
                nxt = spans[(q + 1) % len(ks)][0]
                line += f", last-exit->next first-entry {(nxt - e) * 0.01:.2f} us"
                print(line)
    sv.close()
