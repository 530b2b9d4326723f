#!/usr/bin/env python3
"""Time one relevance-gate encoder pass (HIP BERT-base, graphed buckets) at the gate service's batch
sizes: ``n`` queries of ``L`` tokens packed into one pass, plus the cosine against cached assignment
embeddings.  One JSON line per batch size."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,16,64,127")
    ap.add_argument("--tokens", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    args = ap.parse_args()
    from distributed_lms_raft_llm_amd.gate.relevance import RelevanceGate

    gate = RelevanceGate.create("bert-base-uncased", device="cuda")
    g = torch.Generator().manual_seed(0)
    for n in [int(b) for b in args.batches.split(",")]:
        batch = [torch.randint(1000, 20000, (args.tokens,), generator=g).tolist() for _ in range(n)]
        for _ in range(3):
            gate.encoder.embed(batch)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.reps):
            gate.encoder.embed(batch)
        ev1.record()
        ev1.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        print(json.dumps({"queries": n, "tokens_each": args.tokens, "gpu_ms_per_pass": round(ev0.elapsed_time(ev1) / args.reps, 3),
                          "wall_ms_per_pass": round(wall, 3)}), flush=True)


if __name__ == "__main__":
    main()
