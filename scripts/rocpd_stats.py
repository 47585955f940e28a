#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (run_results.db): calls, total / average
/ min duration (us), grid and block sizes; prints a markdown table, largest total first."""
import sqlite3
import sys


def stats(db, limit=25):
    con = sqlite3.connect(db)
    rows = con.execute(
        "select s.kernel_name, count(*), sum(d.\"end\" - d.start), avg(d.\"end\" - d.start), min(d.\"end\" - d.start), "
        "max(d.grid_size_x), max(d.workgroup_size_x) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
        "on d.kernel_id = s.id group by s.kernel_name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    out = ["| kernel | calls | total us | % | avg us | min us | grid x | block |", "|---|---|---|---|---|---|---|---|"]
    for name, n, t, a, mn, gx, bx in rows[:limit]:
        short = name.split("(")[0][:70]
        out.append(f"| `{short}` | {n} | {t / 1e3:.1f} | {100 * t / tot:.1f} | {a / 1e3:.2f} | {mn / 1e3:.2f} | {gx} | {bx} |")
    return "\n".join(out)


if __name__ == "__main__":
    for db in sys.argv[1:]:
        print(f"### {db}\n")
        print(stats(db))
        print()
