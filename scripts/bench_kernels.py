#!/usr/bin/env python3
"""Per-kernel microbenchmark of the decode hot path (GPT-2 shapes) on one MI355X.

Each measurement captures ``--inner`` back-to-back launches of one kernel into a hipGraph and
times graph replays with events (host launch overhead excluded, inter-kernel boundaries
included -- what the decode graph pays), interleaving variants in one process
(cdna_hip_programming.md §5.4 rule 24) on random data.  GEMM tiles can be forced to sweep the
tile/ring-depth configurations.  Prints one JSON object per measurement and a SUMMARY line.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lms_raft_llm_amd import ops  # noqa: E402

TILES = {-1: "auto", 0: "32x64s6", 1: "64x64s4", 2: "128x64s3", 3: "128x128s3", 4: "64x64s2", 5: "64x128s3",
         6: "128x128s2", 7: "64x64s6", 8: "256x128w8s2", 9: "128x256w8s2", 10: "128x128w8s3(4x2)",
         11: "128x128w8s3(2x4)", 12: "256x128s2(wave128x64)", 13: "256x128s3(wave128x64)",
         14: "256x256w8s2(wave128x64)", 17: "64x96s4", 18: "64x96s3", 19: "64x96s6"}


def graph_time(fn, inner=20, reps=15):
    """``fn(i)`` is launch i of the captured sequence (lets cold-weight runs rotate buffers)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(inner):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--vocab", type=int, default=50304, help="LM-head N (padded vocabulary)")
    ap.add_argument("--batches", default="64,256,512")
    ap.add_argument("--tiles", default="-1,1,2,3,4,5,7")
    ap.add_argument("--T", type=int, default=150)
    ap.add_argument("--cold-mb", type=int, default=768,
                    help="rotate GEMM weights over >= this many MB per graph so they stream from HBM like "
                         "the 12-layer decode step (0: one L2/MALL-hot weight)")
    ap.add_argument("--ops", default="qkv,oproj,fc,proj,lmhead,attn,add_ln")
    ap.add_argument("--vendor", action="store_true", help="also time torch.mm (hipBLASLt) on the same shapes")
    args = ap.parse_args()
    ops_on = set(args.ops.split(","))
    L = ops.lib()
    dev = "cuda"
    d = args.d
    H = d // 64
    V = args.vocab
    tiles = [int(t) for t in args.tiles.split(",")]
    res = []

    def rec(**kw):
        res.append(kw)
        print(json.dumps(kw), flush=True)

    for M in [int(x) for x in args.batches.split(",")]:
        a = torch.randn(M, d, device=dev).to(torch.bfloat16)
        a4 = torch.randn(M, 4 * d, device=dev).to(torch.bfloat16)

        def weights(N, K):
            n = 1 if not args.cold_mb else max(1, min(640, -(-args.cold_mb * 2**20 // (N * K * 2))))
            base = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            return [base] + [base.clone() for _ in range(n - 1)]

        shapes = {
            "qkv": (a, (3 * d, d)), "oproj": (a, (d, d)), "fc": (a, (4 * d, d)), "proj": (a4, (d, 4 * d)),
            "lmhead": (a, (V, d)),
        }
        parts = torch.empty(8, M, d, device=dev)
        keys = torch.zeros(M, V // 64, dtype=torch.int64, device=dev)
        seen = torch.zeros(M, V // 32, dtype=torch.int32, device=dev)
        out_bf = torch.empty(M, V, dtype=torch.bfloat16, device=dev)
        for name, (x, (N, K)) in shapes.items():
            if name not in ops_on:
                continue
            ws = weights(N, K)
            nw = len(ws)
            inner = max(20, nw)
            variants = []
            if name in ("oproj", "proj"):
                for s in (1, 2, 4, 8):
                    if (K // 64) % s == 0:
                        variants.append((f"split{s}", lambda i, x=x, s=s: ops.gemm(x, ws[i % nw], ops.EPI_PARTIAL,
                                                                                   out=parts, split_k=s)))
            elif name == "lmhead":
                variants.append(("argmax", lambda i, x=x: ops.gemm(x, ws[i % nw], ops.EPI_ARGMAX, argmax_out=keys,
                                                                   seen=seen, vocab=50257, penalty=1.2)))
                # same GEMM with a plain bf16 logits store: the fused penalty/argmax epilogue's cost
                variants.append(("bf16_logits", lambda i, x=x, N=N: ops.gemm(x, ws[i % nw], ops.EPI_BF16,
                                                                             out=out_bf[:, :N])))
            else:
                variants.append(("bf16", lambda i, x=x, N=N: ops.gemm(x, ws[i % nw], ops.EPI_BF16, out=out_bf[:, :N])))
            if args.vendor:  # hipBLASLt/rocBLAS via torch, same shapes and weight rotation (reference point)
                variants.append(("torch_mm", lambda i, x=x: torch.mm(x, ws[i % nw].t())))
            for vname, fn in variants:
                for t in (tiles if vname != "torch_mm" else [-1]):
                    L.dlms_gemm_force_tile(t)
                    try:
                        med, mn = graph_time(fn, inner=inner)
                    finally:
                        L.dlms_gemm_force_tile(-1)
                    flops = 2 * M * N * K
                    byts = (M * K + N * K) * 2
                    rec(M=M, op=name, variant=vname, tile=TILES[t], us=round(med, 2), us_min=round(mn, 2),
                        tflops=round(flops / med / 1e6, 1), GBps=round(byts / med / 1e3, 1), weight_copies=nw)
            del ws
        if "attn" not in ops_on and "add_ln" not in ops_on:
            continue
        kc = torch.randn(M, H, args.T, 64, device=dev).to(torch.bfloat16)
        vc = torch.randn(M, H, args.T, 64, device=dev).to(torch.bfloat16)
        q = torch.randn(M, d, device=dev).to(torch.bfloat16)
        slot = torch.arange(M, dtype=torch.int32, device=dev)
        o = torch.empty(M, d, dtype=torch.bfloat16, device=dev)
        for Lk in (32, 90, args.T):
            kvl = torch.full((M,), Lk, dtype=torch.int32, device=dev)
            for impl in ("wave", "persist", "lds"):
                if "attn" not in ops_on:
                    break
                med, mn = graph_time(lambda i, impl=impl: ops.row_attention(q, kc, vc, slot, kvl, out=o, impl=impl))
                byts = M * H * Lk * 64 * 2 * 2
                rec(M=M, op="attn", variant=f"{impl}_T{Lk}", us=round(med, 2), us_min=round(mn, 2),
                    GBps=round(byts / med / 1e3, 1))
        x = torch.randn(M, d, device=dev)
        g = torch.ones(d, device=dev)
        b = torch.zeros(d, device=dev)
        h = torch.empty(M, d, dtype=torch.bfloat16, device=dev)
        for s in (0, 4, 8):
            if "add_ln" not in ops_on:
                break
            med, mn = graph_time(lambda i, s=s: ops.add_layernorm(x, g, b, 1e-5, parts=parts if s else None, nsplit=s,
                                                               bias=b, out_bf16=h))
            rec(M=M, op="add_ln", variant=f"split{s}", us=round(med, 2), us_min=round(mn, 2))
    print("SUMMARY " + json.dumps(res))


if __name__ == "__main__":
    main()
