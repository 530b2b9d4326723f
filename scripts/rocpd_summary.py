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


def gaps(db: str, min_kernels: int = 50):
    """Idle gaps between consecutive kernels on the busiest queue (graph replays): returns
    (kernel_count, busy_us, span_us, median_gap_us) over the longest dense stretch."""
    c = sqlite3.connect(db)
    rows = c.execute("select start, end from kernels order by start").fetchall()
    if len(rows) < min_kernels:
        return None
    g = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    dense = [x for x in g if x < 50]  # ignore host gaps between replays / phases
    dense.sort()
    busy = sum(e - s for s, e in rows) / 1e3
    return len(rows), busy, (rows[-1][1] - rows[0][0]) / 1e3, dense[len(dense) // 2] if dense else None, \
        sum(dense) / max(1, len(dense))
