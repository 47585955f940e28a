#!/usr/bin/env python3
"""Per-kernel active-launch means from rocprofv3 rocpd databases (run_results.db): launches
longer than a threshold (default 20 us) only, so the no-op launches of iterations past an
inner loop's exit inside a batch do not dilute the mean.  argv: db [db ...] [--min US]."""
import collections
import sqlite3
import sys


def active(db, min_us):
    con = sqlite3.connect(db)
    rows = con.execute('select s.kernel_name, d."end" - d.start from rocpd_kernel_dispatch d join '
                       'rocpd_info_kernel_symbol s on d.kernel_id = s.id').fetchall()
    agg = collections.defaultdict(list)
    for name, t in rows:
        agg[name.split("(")[0]].append(t / 1e3)
    out = {}
    for k, v in agg.items():
        act = [x for x in v if x > min_us]
        if act:
            out[k] = (len(act), sum(act) / len(act), sum(act))
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mn = 20.0
    if "--min" in sys.argv:
        mn = float(sys.argv[sys.argv.index("--min") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--min") + 1]]
    res = [active(db, mn) for db in args]
    keys = sorted(set().union(*res), key=lambda k: -max(r.get(k, (0, 0, 0))[2] for r in res))
    print("| kernel | " + " | ".join(f"{db} active / mean us" for db in args) + " |")
    print("|---|" + "---|" * len(args))
    for k in keys[:25]:
        cells = [f"{r[k][0]} / {r[k][1]:.1f}" if k in r else "-" for r in res]
        print(f"| `{k[:60]}` | " + " | ".join(cells) + " |")
