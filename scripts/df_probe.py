#!/usr/bin/env python3
"""Probe of the persistent dataflow decode: correctness against the launch-per-op path on small
configs, then batch-1/2 query latency on a model (prints one JSON line per point)."""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def engine(cfg, w, df: bool, **kw):
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    os.environ["DLMS_DATAFLOW"] = "1" if df else "0"
    os.environ["DLMS_DATAFLOW_ROWS"] = "2"
    return HipGPT2Engine(cfg, w, **kw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--skip-tiny", action="store_true")
    ap.add_argument("--no-ref", action="store_true")
    args = ap.parse_args()
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    if not args.skip_tiny:
        cfg = gpt2_config("gpt2-tiny")
        w = init_gpt2_weights(cfg, seed=0)
        prompts = [[5, 6, 7, 8, 9], [11, 12, 13]]
        for B in (1, 2):
            a = engine(cfg, w, True, max_batch=2, max_length=48)
            t0 = time.perf_counter()
            ra = a.generate(prompts[:B])
            torch.cuda.synchronize()
            rb = engine(cfg, w, False, max_batch=2, max_length=48).generate(prompts[:B])
            print(json.dumps({"probe": "tiny", "B": B, "equal": ra == rb, "df": ra, "ref": rb,
                              "s": round(time.perf_counter() - t0, 3)}), flush=True)
    cfg = gpt2_config(args.model)
    w = init_gpt2_weights(cfg, seed=0)
    g = torch.Generator().manual_seed(1)
    for B in args.batch:
        prompts = torch.randint(0, cfg.vocab_size - 1, (B, args.prompt_len), generator=g).tolist()
        res = {"probe": args.model, "B": B}
        for df in ((True,) if args.no_ref else (True, False)):
            eng = engine(cfg, w, df, max_batch=max(2, B), max_length=args.max_length)
            out = eng.generate(prompts)
            eng.generate(prompts)
            times = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o2 = eng.generate(prompts)
                torch.cuda.synchronize()
                times.append((time.perf_counter() - t0) * 1e3)
            key = "df" if df else "ref"
            res[f"{key}_p50_ms"] = round(statistics.median(times), 3)
            res[f"{key}_min_ms"] = round(min(times), 3)
            res[f"{key}_new_tokens"] = sum(len(o) for o in out) - B * args.prompt_len
            res[f"{key}_stable"] = o2 == out
            res[f"{key}_tokens"] = out[0][args.prompt_len: args.prompt_len + 12]
            del eng
            torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
