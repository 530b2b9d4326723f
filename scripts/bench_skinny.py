#!/usr/bin/env python3
"""Latency-path kernel microbench (GPT-2 decode shapes, M <= 32 rows) on one MI355X.

Times hipGraph replays of ``--inner`` back-to-back launches (inter-kernel boundaries included,
host launch overhead excluded) for the skinny pre-shuffled GEMMs vs the tiled MFMA GEMM, and for
the split-K flash-decode vs the one-wave-per-(row, head) attention.  Weights rotate over >= 512 MB
of copies so they stream from HBM as in a real 12-layer step.  One JSON object per measurement.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lms_raft_llm_amd import ops  # noqa: E402


def graph_time(fn, inner=24, reps=15):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
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
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--batches", default="1,4,16,32")
    ap.add_argument("--attn-only", action="store_true")
    ap.add_argument("--cold-mb", type=int, default=512)
    ap.add_argument("--T", default="150,1024")
    args = ap.parse_args()
    dev = "cuda"
    D = args.d
    shapes = {"qkv": (3 * D, D), "oproj": (D, D), "fc": (4 * D, D), "proj": (D, 4 * D), "lmhead": (50304, D)}
    for M in [int(m) for m in args.batches.split(",")]:
        for op, (N, K) in ({} if args.attn_only else shapes).items():
            copies = max(1, min(24, args.cold_mb * (1 << 20) // (N * K * 2)))
            ws = [torch.randn(N, K, device=dev).mul_(0.02).to(torch.bfloat16) for _ in range(copies)]
            wsh = [ops.shuffle_weight(w) for w in ws]
            bias = torch.randn(N, device=dev)
            res = {}
            if op in ("qkv", "fc"):
                x = torch.randn(M, K, device=dev)
                g, b = torch.ones(K, device=dev), torch.zeros(K, device=dev)
                h = torch.randn(M, K, device=dev).to(torch.bfloat16)
                epi = ops.EPI_GELU_TANH if op == "fc" else ops.EPI_BF16
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                if M <= ops.SKINNY_MAX_M:
                    res["skinny_ln"] = graph_time(lambda i: ops.skinny_gemm(x, wsh[i % copies], epi, ln=(g, b, 1e-5),
                                                                         bias=bias, out=out))
                res["tiled+ln"] = graph_time(lambda i: (ops.layernorm(x, g, b, 1e-5, out_bf16=h),
                                                        ops.gemm(h, ws[i % copies], epi, bias=bias, out=out)))
                if M > 1 and M <= ops.mid_max_rows(K):  # mid.hip: the 9-64-row fused LN + GEMM, per geometry
                    for geo in (1, 2, 3, 4, 5, 6, 7):
                        try:
                            res[f"mid_ln_g{geo}"] = graph_time(
                                lambda i, geo=geo: ops.mid_ln_gemm(x, wsh[i % copies], epi, g, b, 1e-5, bias=bias,
                                                                   out=out, geo=geo))
                        except RuntimeError:
                            pass
            elif op in ("oproj", "proj"):
                a = torch.randn(M, K, device=dev).to(torch.bfloat16)
                x = torch.randn(M, N, device=dev)
                if M <= ops.SKINNY_MAX_M:
                    res["skinny_resid"] = graph_time(lambda i: ops.skinny_gemm(a, wsh[i % copies], ops.EPI_F32, bias=bias,
                                                                            out=x))
                if M > 1:  # mid.hip's in-place projection, per geometry
                    for geo in (1, 2, 3, 4, 5, 6):
                        try:
                            res[f"mid_proj_g{geo}"] = graph_time(
                                lambda i, geo=geo: ops.mid_proj(a, wsh[i % copies], x, bias=bias, geo=geo))
                        except RuntimeError:
                            pass
                parts = torch.empty(8, M, N, device=dev)
                res["tiled_split4"] = graph_time(lambda i: ops.gemm(a, ws[i % copies], ops.EPI_PARTIAL, out=parts,
                                                                    split_k=4))
            else:
                h = torch.randn(M, K, device=dev).to(torch.bfloat16)
                keys = torch.zeros(M, N // 64, dtype=torch.int64, device=dev)
                seen = torch.zeros(M, N // 32, dtype=torch.int32, device=dev)
                if M <= ops.SKINNY_MAX_M:
                    res["skinny_argmax"] = graph_time(lambda i: ops.skinny_gemm(h, wsh[i % copies], ops.EPI_ARGMAX,
                                                                             argmax_out=keys, seen=seen, vocab=50257,
                                                                             penalty=1.2))
                res["tiled_argmax"] = graph_time(lambda i: ops.gemm(h, ws[i % copies], ops.EPI_ARGMAX, argmax_out=keys,
                                                                    seen=seen, vocab=50257, penalty=1.2))
            for k, (med, mn) in res.items():
                print(json.dumps({"M": M, "op": op, "variant": k, "us": round(med, 2), "us_min": round(mn, 2),
                                  "GBps": round(N * K * 2 / med / 1e3, 1)}), flush=True)
            del ws, wsh
        H = D // 64
        for T in [int(t) for t in args.T.split(",")]:
            S = max(M, 1)
            nrot = max(1, min(16, args.cold_mb * (1 << 20) // (S * H * T * 64 * 2 * 2)))
            caches = [(torch.randn(S, H, T, 64, device=dev).to(torch.bfloat16),
                       torch.randn(S, H, T, 64, device=dev).to(torch.bfloat16)) for _ in range(nrot)]
            q = torch.randn(M, D, device=dev).to(torch.bfloat16)
            slot = torch.arange(M, dtype=torch.int32, device=dev)
            kvlen = torch.full((M,), T, dtype=torch.int32, device=dev)
            out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
            kv_bytes = M * H * T * 64 * 2 * 2
            res = {"wave": graph_time(lambda i: ops.row_attention(q, *caches[i % nrot], slot, kvlen, out=out))}
            for nw in (4, 8, 16):
                res[f"split{nw}"] = graph_time(lambda i: ops.attention_split(q, *caches[i % nrot], slot, kvlen, out=out,
                                                                             waves=nw))
            geo = ops.attention_split_geometry(M * H, T)
            wsp = ops.AttnSplitWorkspace(M * H, 64, dev)
            for nw, ns in sorted({(4, 2), (4, 4), (4, 8), (2, 8), (8, 4), (4, 16), geo}):
                if ns > 1:
                    res[f"splitwg{nw}x{ns}" + ("*" if (nw, ns) == geo else "")] = graph_time(
                        lambda i: ops.attention_split(q, *caches[i % nrot], slot, kvlen, out=out, waves=nw, splits=ns,
                                                      workspace=wsp))
            for k, (med, mn) in res.items():
                print(json.dumps({"M": M, "op": f"attn_T{T}", "variant": k, "us": round(med, 2), "us_min": round(mn, 2),
                                  "GBps": round(kv_bytes / med / 1e3, 1)}), flush=True)
            del caches


if __name__ == "__main__":
    main()
