#!/usr/bin/env python3
"""Open-loop serving benchmark of the tutoring path on one MI355X: Poisson query arrivals at
``--rate`` queries/s into the continuous batcher (engine/scheduler.py) or the window batcher
(tutor/server.py), GPT-2-124M, prompt ``--prompt-len`` tokens -> max_length 150, greedy +
repetition penalty 1.2.  Reports per-query latency percentiles and delivered tokens/s as JSON
lines (one per mode and rate).

Synthetic prompts (random token ids) and random-init weights: no checkpoint on this box.
"""
import argparse
import json
import os
import random
import statistics
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine  # noqa: E402
from distributed_lms_raft_llm_amd.engine.scheduler import ContinuousBatcher  # noqa: E402
from distributed_lms_raft_llm_amd.models.config import GenerationConfig, gpt2_config  # noqa: E402
from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights  # noqa: E402
from distributed_lms_raft_llm_amd.tutor.server import Batcher  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def run_load(submit, prompts, rate, seed=0):
    """Open loop: query i is issued at its Poisson arrival time regardless of completions."""
    rng = random.Random(seed)
    lat = [None] * len(prompts)
    toks = [0] * len(prompts)
    done = threading.Semaphore(0)
    t0 = time.perf_counter()
    t_next = t0
    for i, p in enumerate(prompts):
        t_next += rng.expovariate(rate)
        d = t_next - time.perf_counter()
        if d > 0:
            time.sleep(d)
        ts = time.perf_counter()
        f = submit(p)

        def cb(fut, i=i, ts=ts, n=len(p)):
            lat[i] = (time.perf_counter() - ts) * 1e3
            toks[i] = len(fut.result()) - n
            done.release()

        f.add_done_callback(cb)
    for _ in prompts:
        done.acquire()
    wall = time.perf_counter() - t0
    return lat, sum(toks), wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--rates", default="200,1000", help="queries per second (Poisson), comma list")
    ap.add_argument("--queries", type=int, default=2000)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--prompt-jitter", type=int, default=16)
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--modes", default="continuous,window")
    ap.add_argument("--chunk", type=int, default=8)
    ap.add_argument("--window-ms", type=float, default=5.0)
    args = ap.parse_args()

    cfg = gpt2_config(args.model)
    w = init_gpt2_weights(cfg, seed=0)
    eng = HipGPT2Engine(cfg, w, max_batch=args.max_batch, max_length=args.max_length)
    rng = random.Random(1)
    prompts = [[rng.randrange(cfg.vocab_size - 1)
                for _ in range(max(1, args.prompt_len + rng.randint(-args.prompt_jitter, args.prompt_jitter)))]
               for _ in range(args.queries)]
    for mode in args.modes.split(","):
        for rate in [float(r) for r in args.rates.split(",")]:
            if mode == "continuous":
                b = ContinuousBatcher(eng, 1.2, chunk=args.chunk)
            else:
                b = Batcher(eng, GenerationConfig(max_length=args.max_length, repetition_penalty=1.2),
                            max_batch=args.max_batch, window_ms=args.window_ms)
            run_load(b.submit, prompts[: min(300, len(prompts))], rate=rate * 4)  # warm graphs/buckets
            torch.cuda.synchronize()
            lat, toks, wall = run_load(b.submit, prompts, rate=rate)
            b.stop()
            print(json.dumps({"mode": mode, "rate_qps": rate, "queries": len(prompts), "tokens_per_s": round(toks / wall, 1),
                              "p50_ms": round(statistics.median(lat), 2), "p90_ms": round(pct(lat, 0.9), 2),
                              "p99_ms": round(pct(lat, 0.99), 2), "mean_ms": round(statistics.fmean(lat), 2),
                              "wall_s": round(wall, 2), "max_batch": args.max_batch, "model": args.model,
                              "max_length": args.max_length}), flush=True)


if __name__ == "__main__":
    main()
