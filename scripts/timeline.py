#!/usr/bin/env python3
"""Critical-path view of one overlapped decode step from a rocprofv3 kernel trace: per hardware
queue, which kernel families run when, how long attention and the GEMM-side chain overlap, and the
idle gaps.  usage: timeline.py <kernel_trace.csv>

Caveat (measured): under rocprofv3 --kernel-trace the overlapped step ran at 2150 us vs 1490 us
unprofiled and the two queues barely overlapped (profiles/r2_timeline_b1024_profiled.txt), so the
tracer itself serialises much of the concurrency; forcing the attentions to alternate between the
queues (the since-removed alternating-attention schedule) was 4 % SLOWER unprofiled (profiles/r2_sweep_alt_attn.jsonl)."""
import csv
import sys
from collections import defaultdict


def family(name: str) -> str:
    for key, fam in (("attn", "attention"), ("gemm_ps", "lm_head"), ("gemm_tn", "gemm"), ("skinny", "gemm"),
                     ("layernorm", "layernorm"), ("decode_update", "update"), ("embed", "embed")):
        if key in name:
            return fam
    return "other"


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]))
    rows.sort()
    # decode steps end with decode_update on each queue; take the steps of the timed generation
    ups = [i for i, r in enumerate(rows) if "decode_update" in r[3]]
    if len(ups) < 20:
        print("too few decode steps in trace")
        return
    # pick a window of 10 steps from the middle of the last generation (2 updates per step: halves)
    mid = ups[len(ups) - 120]
    end = ups[len(ups) - 100]
    win = [r for r in rows if rows[mid][1] <= r[0] and r[1] <= rows[end][1]]
    t0, t1 = min(r[0] for r in win), max(r[1] for r in win)
    span = (t1 - t0) / 1e3
    busy = defaultdict(float)
    per_q = defaultdict(float)
    events = []
    for s, e, q, n in win:
        fam = family(n)
        busy[fam] += (e - s) / 1e3
        per_q[q] += (e - s) / 1e3
        events.append((s, 1, fam))
        events.append((e, -1, fam))
    events.sort()
    active = defaultdict(int)
    last = t0
    both = attn_only = other_only = idle = 0.0
    for t, d, fam in events:
        dt = (t - last) / 1e3
        a = active["attention"] > 0
        o = sum(v for k, v in active.items() if k != "attention") > 0
        if a and o:
            both += dt
        elif a:
            attn_only += dt
        elif o:
            other_only += dt
        else:
            idle += dt
        active[fam] += d
        last = t
    steps = 10
    print(f"window: {steps} decode steps, {span:.1f} us ({span / steps:.1f} us/step), {len(win)} kernels")
    for fam, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"  {fam:10s} kernel time {v / steps:8.1f} us/step")
    for q, v in sorted(per_q.items()):
        print(f"  queue {q}: busy {v / steps:.1f} us/step")
    print(f"  attention + other concurrently {both / steps:.1f} us/step, attention alone {attn_only / steps:.1f}, "
          f"other alone {other_only / steps:.1f}, idle {idle / steps:.1f}")


if __name__ == "__main__":
    main()
