#!/usr/bin/env python3
"""Per-kernel hardware-counter summary from rocprofv3 ``--pmc`` CSV output (one or more
``*counter_collection.csv`` files, one per pass): mean counter value per dispatch, mean duration,
and derived rates (HBM-side bytes/us, MFMA-busy and wait fractions).
usage: pmc_summary.py out.json file1.csv [file2.csv ...]"""
import csv
import json
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")[:90]


def main():
    out, files = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    dur[k][(f, r.get("Dispatch_Id"))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    res = {}
    for k, cs in vals.items():
        d = {c: round(sum(v) / len(v), 1) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        ds = list(dur[k].values())
        if ds:
            d["avg_us"] = round(sum(ds) / len(ds), 2)
        if "FETCH_SIZE" in d and d.get("avg_us"):
            d["fetch_GBps"] = round(d["FETCH_SIZE"] * 1024 / d["avg_us"] / 1e3, 1)  # FETCH_SIZE is in KB
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            d["wait_frac"] = round(d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"], 3)
            d["active_frac"] = round(d.get("SQ_ACTIVE_INST_ANY", 0) / d["SQ_WAVE_CYCLES"], 3)
        if "SQ_BUSY_CYCLES" in d and d["SQ_BUSY_CYCLES"]:
            d["mfma_busy_per_busy_cycle"] = round(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / d["SQ_BUSY_CYCLES"], 3)
        res[k] = d
    res = dict(sorted(res.items(), key=lambda kv: -kv[1].get("avg_us", 0) * kv[1]["dispatches"]))
    json.dump(res, open(out, "w"), indent=1)
    for k, d in list(res.items())[:12]:
        print(k[:60], {x: d.get(x) for x in ("dispatches", "avg_us", "fetch_GBps", "wait_frac", "mfma_busy_per_busy_cycle")})


if __name__ == "__main__":
    main()
