#!/usr/bin/env python3
"""Per-kernel microbenchmark of the decode hot path (GPT-2 shapes) on one MI355X.

Times every kernel shape the decode step launches, in one process with interleaved repetitions
(cdna_hip_programming.md §5.4 rule 24), on random data, and prints a JSON summary with achieved
TFLOP/s and GB/s (unique bytes) per shape.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lms_raft_llm_amd import ops  # noqa: E402


def timeit(fn, reps=50, inner=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(inner):
            fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--batches", default="64,256,512")
    ap.add_argument("--T", type=int, default=150)
    args = ap.parse_args()
    dev = "cuda"
    d = args.d
    H = d // 64
    V = 50304
    res = []
    for M in [int(x) for x in args.batches.split(",")]:
        a = torch.randn(M, d, device=dev).to(torch.bfloat16)
        a4 = torch.randn(M, 4 * d, device=dev).to(torch.bfloat16)
        shapes = {
            "qkv": (a, torch.randn(3 * d, d, device=dev).to(torch.bfloat16) * 0.02),
            "oproj": (a, torch.randn(d, d, device=dev).to(torch.bfloat16) * 0.02),
            "fc": (a, torch.randn(4 * d, d, device=dev).to(torch.bfloat16) * 0.02),
            "proj": (a4, torch.randn(d, 4 * d, device=dev).to(torch.bfloat16) * 0.02),
            "lmhead": (a, torch.randn(V, d, device=dev).to(torch.bfloat16) * 0.02),
        }
        parts = torch.empty(8, M, d, device=dev)
        keys = torch.zeros(M, dtype=torch.int64, device=dev)
        seen = torch.zeros(M, V // 32, dtype=torch.int32, device=dev)
        out_bf = torch.empty(M, 4 * d, dtype=torch.bfloat16, device=dev)
        for name, (x, w) in shapes.items():
            N, K = w.shape
            variants = []
            if name in ("oproj", "proj"):
                for s in (1, 2, 4, 8):
                    if (K // 64) % s == 0:
                        variants.append((f"split{s}", lambda x=x, w=w, s=s: ops.gemm(x, w, ops.EPI_PARTIAL, out=parts,
                                                                                   split_k=s)))
            elif name == "lmhead":
                variants.append(("argmax", lambda x=x, w=w: ops.gemm(x, w, ops.EPI_ARGMAX, argmax_out=keys, seen=seen,
                                                                     vocab=50257, penalty=1.2)))
            else:
                variants.append(("bf16", lambda x=x, w=w, N=N: ops.gemm(x, w, ops.EPI_BF16, out=out_bf[:, :N])))
            for vname, fn in variants:
                med, mn = timeit(fn)
                flops = 2 * M * N * K
                byts = (M * K + N * K) * 2
                res.append({"M": M, "op": name, "variant": vname, "us": round(med, 2), "us_min": round(mn, 2),
                            "tflops": round(flops / med / 1e6, 1), "GBps": round(byts / med / 1e3, 1)})
                print(json.dumps(res[-1]), flush=True)
        # attention over a full-length cache
        kc = torch.randn(M, H, args.T, 64, device=dev).to(torch.bfloat16)
        vc = torch.randn(M, H, args.T, 64, device=dev).to(torch.bfloat16)
        q = torch.randn(M, d, device=dev).to(torch.bfloat16)
        slot = torch.arange(M, dtype=torch.int32, device=dev)
        for L in (32, 90, args.T):
            kvl = torch.full((M,), L, dtype=torch.int32, device=dev)
            o = torch.empty(M, d, dtype=torch.bfloat16, device=dev)
            med, mn = timeit(lambda: ops.row_attention(q, kc, vc, slot, kvl, out=o))
            byts = M * H * L * 64 * 2 * 2
            res.append({"M": M, "op": "attn", "variant": f"T{L}", "us": round(med, 2), "us_min": round(mn, 2),
                        "GBps": round(byts / med / 1e3, 1)})
            print(json.dumps(res[-1]), flush=True)
        x = torch.randn(M, d, device=dev)
        g = torch.ones(d, device=dev)
        b = torch.zeros(d, device=dev)
        h = torch.empty(M, d, dtype=torch.bfloat16, device=dev)
        for s in (0, 4, 8):
            med, mn = timeit(lambda s=s: ops.add_layernorm(x, g, b, 1e-5, parts=parts if s else None, nsplit=s,
                                                           bias=b, out_bf16=h))
            res.append({"M": M, "op": "add_ln", "variant": f"split{s}", "us": round(med, 2), "us_min": round(mn, 2)})
            print(json.dumps(res[-1]), flush=True)
    print("SUMMARY " + json.dumps(res))


if __name__ == "__main__":
    main()
