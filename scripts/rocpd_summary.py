#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max us, % of GPU time) from a rocprofv3 rocpd SQLite
database (ROCm 7 default output).  usage: rocpd_summary.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys


def summarize(db: str):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(n, cnt, tot / 1e3, avg / 1e3, mn / 1e3, mx / 1e3, 100.0 * tot / total) for n, cnt, tot, avg, mn, mx in rows]


if __name__ == "__main__":
    rows = summarize(sys.argv[1])
    out = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    out.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
    for r in rows:
        out.writerow([r[0][:140], r[1]] + [round(x, 2) for x in r[2:]])
