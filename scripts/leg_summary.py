#!/usr/bin/env python3
"""Summarise one scripts/leg_profile.sh leg: per-stage and per-kernel rocprofv3 figures over the
FULL launches of lrs_time_stages / lrs_time_auut only (scripts/leg_probe.py), and the HBM-side
bytes per launch from the separate FETCH_SIZE / WRITE_SIZE passes.

The kernel trace is split on the probe's idle gaps (> 100 ms) into
  [priming iteration] [stage A x reps] ([stage G x reps]) [stage B x reps] [A(UU^T) x reps]
so every kernel is attributed to the stage whose relaunch loop issued it, and no launch of the
warmup solve (nor any no-op launch after an inner loop's exit) enters a mean.  The counter
passes carry no timestamps: their dispatches are aligned with the trace's from the end of the
run (same program, same dispatch sequence; kernel names are checked position by position).

FETCH_SIZE is doubled (MI355X_MICROARCH.md "HBM": gfx950 reports half the bytes of a wide
coalesced read); WRITE_SIZE is taken as reported.  Both are KB per dispatch in the CSVs.

usage: leg_summary.py <leg dir> <tag> -> <leg dir>/<tag>_summary.md, <tag>_pmc.json"""
import collections
import csv
import glob
import json
import os
import sys

GAP_NS = 100e6


def clean(name):
    return name.split("(")[0].replace("void ", "").strip()


def base(name):
    return clean(name).split("<")[0].split("::")[-1]


def trace_rows(d):
    f = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    rows.sort()
    return rows


def counter_rows(d, sub, counter):
    fs = glob.glob(os.path.join(d, sub, "*counter_collection.csv"))
    if not fs:
        return None
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(fs[0])):
        if r["Counter_Name"] != counter:
            continue
        k = int(r["Dispatch_Id"])
        per[k] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"]
    return [(names[k], per[k]) for k in sorted(per)]


def main():
    d, tag = sys.argv[1], sys.argv[2]
    probe = None
    for ln in open(os.path.join(d, "trace.log")):
        if ln.startswith("{\"leg\""):
            probe = json.loads(ln)
    reps = probe["reps"]
    rows = trace_rows(d)
    segs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if b[0] - a[1] > GAP_NS:
            segs.append(cur)
            cur = []
        cur.append(b)
    segs.append(cur)
    has_g = probe["stage_us"][1] > 0
    names = ["A", "G", "B", "auut"] if has_g else ["A", "B", "auut"]
    tail = segs[-len(names):]
    region = [x for s in tail for x in s]
    stage_of = {}
    lines = [f"# rocprofv3 leg summary `{tag}` ({probe['leg']})", "",
             f"Command: `scripts/leg_profile.sh {tag} {probe['leg']}` -> `scripts/leg_probe.py {probe['leg']} {reps}` "
             "(kernel trace, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes).  Only the launches of the "
             f"timed relaunch loops count: lrs_time_stages ({reps} back-to-back relaunches per stage) and "
             f"lrs_time_auut ({reps}), split on the probe's idle gaps; the warmup solve and the priming iteration "
             "are excluded.", "",
             f"Probe line (HIP events on the solver stream): `{json.dumps(probe)}`", ""]
    # per-kernel per-launch duration (sum over the stage loop / reps) and dispatch counts
    kern = collections.OrderedDict()
    for sname, seg in zip(names, tail):
        for s, e, k in seg:
            key = (sname, clean(k))
            kern.setdefault(key, []).append((e - s) / 1e3)
            stage_of[clean(k)] = sname
    # counters aligned from the end of the run
    pmc = {}
    for sub, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        cr = counter_rows(d, sub, cname)
        if not cr:
            continue
        if len(cr) < len(region):
            print(f"{cname}: {len(cr)} dispatches < {len(region)} in the region", file=sys.stderr)
            continue
        al = cr[-len(region):]
        bad = sum(1 for (kn, _), (_, _, tk) in zip(al, region) if clean(kn) != clean(tk))
        if bad:
            print(f"{cname}: {bad} of {len(region)} aligned dispatches differ in kernel name", file=sys.stderr)
            continue
        i = 0
        for sname, seg in zip(names, tail):
            for s, e, k in seg:
                pmc.setdefault((sname, clean(k)), {}).setdefault(cname, []).append(al[i][1] * 1024.0)
                i += 1
    lines += ["| stage | kernel | launches | per launch us (sum / reps) | median us | max us | "
              "FETCH x2 MB / launch | WRITE MB / launch |", "|---|---|---|---|---|---|---|---|"]
    stage_sum = collections.defaultdict(lambda: [0.0, 0.0, 0.0, True])
    out = {}
    for (sname, k), v in kern.items():
        per = sum(v) / reps
        vs = sorted(v)
        f = pmc.get((sname, k), {}).get("FETCH_SIZE")
        w = pmc.get((sname, k), {}).get("WRITE_SIZE")
        fb = 2 * sum(f) / reps if f else None
        wb = sum(w) / reps if w else None
        ss = stage_sum[sname]
        ss[0] += per
        if fb is None or wb is None:
            ss[3] = False
        else:
            ss[1] += fb
            ss[2] += wb
        lines.append(f"| {sname} | `{k[:70]}` | {len(v)} | {per:.2f} | {vs[len(vs) // 2]:.2f} | {vs[-1]:.2f} | "
                     + (f"{fb / 1e6:.3f}" if fb is not None else "-") + " | "
                     + (f"{wb / 1e6:.3f}" if wb is not None else "-") + " |")
        out[k] = {"stage": sname, "launches": len(v), "per_launch_us": per,
                  "fetch_bytes": fb, "write_bytes": wb, "source": f"profiles/{tag}_summary.md"}
    ev = dict(zip(["A", "G", "B"], probe["stage_us"]))
    ev["auut"] = probe["auut_us"]
    alg = dict(zip(["A", "G", "B"], probe["stage_bytes"]))
    alg["auut"] = probe["auut_bytes"]
    lines += ["", "| stage | rocprof kernel sum us / launch | HIP-event us / launch (probe) | ratio | algorithmic MB | "
              "counter MB (FETCH x2 + WRITE) | counter / algorithmic | algorithmic GB/s at rocprof time | of 8 TB/s |",
              "|---|---|---|---|---|---|---|---|---|"]
    stages = {}
    for sname in names:
        t, fb, wb, ok = stage_sum[sname]
        tr = fb + wb if ok else None
        gbs = alg[sname] / (t * 1e-6) / 1e9 if t > 0 else 0
        stages[sname] = {"rocprof_us": t, "event_us": ev[sname], "algorithmic_bytes": alg[sname],
                         "traffic_bytes": tr, "algorithmic_GBs_rocprof": gbs, "frac_rocprof": gbs / 8000.0}
        lines.append(f"| {sname} | {t:.2f} | {ev[sname]:.2f} | {t / ev[sname] if ev[sname] else 0:.3f} | "
                     f"{alg[sname] / 1e6:.3f} | " + (f"{tr / 1e6:.3f} | {tr / alg[sname]:.3f}" if tr else "- | -")
                     + f" | {gbs:.0f} | {gbs / 8000.0:.3f} |")
    out["_stages"] = stages
    out["_probe"] = probe
    open(os.path.join(d, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(d, f"{tag}_pmc.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
