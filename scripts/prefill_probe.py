#!/usr/bin/env python3
"""Batch-1 prefill probe: GPU-event time (what bench.py reports as ``prefill_ms_b1``) against the
host time spent issuing the prefill, per call, for the engine as bench.py builds it.

    python scripts/prefill_probe.py [--max-batch 1024] [--reps 8]  -> one JSON line

A GPU-event window larger than its kernels means the GPU idled while the host was still issuing
(the events bracket host work); the host column says how much of it that was."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--max-batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--warm-batch", type=int, default=0, help="first run generations at this batch (bench.py order)")
    args = ap.parse_args()
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import GenerateStats, HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    torch.cuda.set_device(0)
    cfg = gpt2_config(args.model)
    eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=args.max_batch, max_length=150)
    if args.warm_batch:
        gw = torch.Generator().manual_seed(1000)
        big = torch.randint(0, cfg.vocab_size - 1, (args.warm_batch, 32), generator=gw).tolist()
        for _ in range(3):
            eng.generate(big, 150)
        torch.cuda.synchronize()
    g = torch.Generator().manual_seed(2000)
    prompts = torch.randint(0, cfg.vocab_size - 1, (args.batch, 32), generator=g).tolist()
    for _ in range(2):
        eng.generate(prompts, 150)
    B = args.batch
    gpu_ms, host_ms, gen_ms, pre_idle_ms = [], [], [], []
    orig = eng._prefill

    def timed_prefill(p, b, pen):
        t0 = time.perf_counter()
        orig(p, b, pen)
        host_ms.append((time.perf_counter() - t0) * 1e3)

    eng._prefill = timed_prefill
    for _ in range(args.reps):
        st = GenerateStats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(prompts, 150, stats=st)
        torch.cuda.synchronize()
        gen_ms.append((time.perf_counter() - t0) * 1e3)
        gpu_ms.append(st.prefill_ms)
    # the prefill alone, synchronised on both sides (device time of its kernels + launch)
    for _ in range(args.reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(prompts, B, 1.2)
        e1.record()
        torch.cuda.synchronize()
        pre_idle_ms.append(e0.elapsed_time(e1))
    env = {k: v for k, v in os.environ.items() if k.startswith("DLMS_")}
    print(json.dumps({"model": args.model, "batch": B, "max_batch": args.max_batch, "warm_batch": args.warm_batch, "env": env,
                      "prefill_gpu_ms_p50": round(statistics.median(gpu_ms), 3),
                      "prefill_gpu_ms": [round(x, 3) for x in gpu_ms],
                      "prefill_host_ms_p50": round(statistics.median(host_ms[-args.reps:]), 3),
                      "prefill_alone_ms_p50": round(statistics.median(pre_idle_ms), 3),
                      "generate_ms_p50": round(statistics.median(gen_ms), 3),
                      "dataflow": eng._df is not None}), flush=True)


if __name__ == "__main__":
    main()
