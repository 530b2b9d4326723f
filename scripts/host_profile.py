#!/usr/bin/env python3
"""Host-side profile of HipGPT2Engine.generate at the bench operating point: wall time against the
GPU-event prefill + decode windows, and the top host functions (cProfile, own time).

    python scripts/host_profile.py [--batch 1024] [--reps 3]  -> text on stdout"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import GenerateStats, HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    torch.cuda.set_device(0)
    cfg = gpt2_config("gpt2")
    eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=args.batch, max_length=150)
    g = torch.Generator().manual_seed(1000)
    prompts = torch.randint(0, cfg.vocab_size - 1, (args.batch, 32), generator=g).tolist()
    for _ in range(2):
        eng.generate(prompts, 150)
    torch.cuda.synchronize()
    walls, gpu = [], []
    prof = cProfile.Profile()
    for _ in range(args.reps):
        st = GenerateStats()
        t0 = time.perf_counter()
        prof.enable()
        eng.generate(prompts, 150, stats=st)
        prof.disable()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        gpu.append(st.prefill_ms + st.decode_ms)
    print("wall ms per generate:", [round(w, 2) for w in walls])
    print("prefill+decode GPU-event ms:", [round(x, 2) for x in gpu])
    print("host-only ms:", [round(w - x, 2) for w, x in zip(walls, gpu)], flush=True)
    pstats.Stats(prof).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
