#!/usr/bin/env python3
"""Median per-phase microseconds over the layers of one or more df_trace.py JSON files, side by
side (layer 0 excluded: its residual edge is the embedding):

    python scripts/df_trace_summary.py profiles/r3_df_trace_g200_gs2.json gpurun_out/dftrace_j4.json
"""
import json
import statistics
import sys


def main(paths):
    cols = []
    keys = None
    for p in paths:
        d = json.load(open(p))
        rows = d["layers"][1:]
        keys = keys or [k for k in rows[0] if k != "layer"]
        med = {k: statistics.median([r[k] for r in rows if r.get(k) is not None]) for k in keys}
        med.update({f"lm.{k}": v for k, v in d.get("lm", {}).items() if isinstance(v, (int, float))})
        cols.append(med)
    allk = keys + sorted({k for c in cols for k in c if k.startswith("lm.")})
    w = max(len(k) for k in allk)
    print(" " * w, *[f"{p.rsplit('/', 1)[-1][:18]:>18}" for p in paths])
    for k in allk:
        print(f"{k:<{w}}", *[f"{c.get(k, float('nan')):>18.2f}" for c in cols])


if __name__ == "__main__":
    main(sys.argv[1:])
