#!/usr/bin/env python3
"""Tensor-parallel decode on ONE GPU: W ranks share cuda:0 (gloo for setup, the one-shot xGMI
peer-memory kernels for every collective, hipGraph-captured decode steps) -- the per-rank kernel
sequence of BASELINE configs 4 / 5 (GPT-2-large TP=4, GPT-2-XL TP=8) on a box that has a single
MI355X.  The 8-GPU run is the driver's; this shows what each rank launches (run it under
``rocprofv3 --kernel-trace --stats``: the parent never touches the GPU, it only starts the ranks)
and the per-query latency of the shared-GPU rehearsal (not a TP speed number: W ranks time-share
one device).

    python scripts/tp_shared_gpu.py --model gpt2-large --tp 4 --batch 1 --reps 3
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(args):
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine
    from distributed_lms_raft_llm_amd.models.config import gpt2_config
    from distributed_lms_raft_llm_amd.models.gpt2 import init_gpt2_weights

    cfg = gpt2_config(args.model)
    eng = HipGPT2Engine(cfg, init_gpt2_weights(cfg, seed=0), max_batch=max(8, args.batch), max_length=args.max_length,
                        tp_group=dist.group.WORLD, use_graph=True, p2p=True)
    g = torch.Generator().manual_seed(1)
    prompts = torch.randint(0, cfg.vocab_size - 1, (args.batch, args.prompt_len), generator=g).tolist()
    for _ in range(2):
        eng.generate(prompts)
    times = []
    for _ in range(args.reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.generate(prompts)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    eng.xgmi.check()
    line = {"rank": rank, "tp": world, "model": args.model, "batch": args.batch,
            "p50_ms_shared_gpu": round(statistics.median(times), 2), "new_tokens": sum(len(o) for o in out) -
            args.batch * args.prompt_len, "tp_fused": eng.tp_fused, "tp_fused_steps": eng.tp_fused_steps,
            "prefill_graphs": sum(1 for st in eng._pgraphs.values() if st["graph"] is not None),
            "layers": cfg.n_layer}
    print(json.dumps(line), flush=True)
    dist.barrier()
    eng.xgmi.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-large")
    ap.add_argument("--tp", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--max-length", type=int, default=150)
    ap.add_argument("--prompt-len", type=int, default=32)
    args = ap.parse_args()
    if "RANK" in os.environ:
        return rank_main(args)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.tp):  # started before this process touches the GPU (it never does)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.tp), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r and not rc:
                rc = r
                for q in procs:
                    q.terminate()
        time.sleep(0.2)
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
