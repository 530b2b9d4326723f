#!/usr/bin/env python3
"""Throughput-path GEMM microbench: gemm_ps (LDS-resident activation panel, pre-shuffled weights
in registers) vs the tiled LDS-DMA gemm at the decode shapes of GPT-2-small, M = 256..1024.
hipGraph replays of back-to-back launches over >= 512 MB of rotating weight copies."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_lms_raft_llm_amd import ops  # noqa: E402
from scripts.bench_skinny import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--batches", default="256,512,1024")
    ap.add_argument("--cold-mb", type=int, default=512)
    ap.add_argument("--ops", default="qkv,fc,oproj,proj,lmhead")
    ap.add_argument("--tiles", default="", help="forced tiled-GEMM configs to time too (dlms_gemm_force_tile ids)")
    args = ap.parse_args()
    forced = [int(t) for t in args.tiles.split(",") if t.strip()]
    L = ops.lib()
    dev, D = "cuda", args.d
    shapes = {"qkv": (3 * D, D, ops.EPI_QKV), "fc": (4 * D, D, ops.EPI_GELU_TANH), "oproj": (D, D, ops.EPI_PARTIAL),
              "proj": (D, 4 * D, ops.EPI_PARTIAL), "lmhead": (50304, D, ops.EPI_ARGMAX)}
    H = D // 64
    for M in [int(m) for m in args.batches.split(",")]:
        for op, (N, K, epi) in shapes.items():
            if op not in args.ops.split(","):
                continue
            copies = max(1, min(24, args.cold_mb * (1 << 20) // (N * K * 2)))
            ws = [torch.randn(N, K, device=dev).mul_(0.02).to(torch.bfloat16) for _ in range(copies)]
            wsh = [ops.shuffle_weight(w) for w in ws]
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            bias = torch.randn(N, device=dev)
            kw, kt = {}, {}
            if epi == ops.EPI_QKV:
                q = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
                kc = torch.zeros(M, H, 152, 64, device=dev, dtype=torch.bfloat16)
                vc = torch.zeros_like(kc)
                slot = torch.arange(M, dtype=torch.int32, device=dev)
                pos = torch.full((M,), 100, dtype=torch.int32, device=dev)
                kw = kt = dict(bias=bias, q_out=q, k_cache=kc, v_cache=vc, row_slot=slot, row_pos=pos)
            elif epi == ops.EPI_GELU_TANH:
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                kw = kt = dict(bias=bias, out=out)
            elif epi == ops.EPI_PARTIAL:
                parts = torch.empty(8, M, N, device=dev)
                kw = dict(out=parts)
                kt = dict(out=parts)
            else:
                seen = torch.zeros(M, N // 32, dtype=torch.int32, device=dev)
                keys = torch.zeros(M, max(N // 64, ops.gemm_ps_key_slots(M, N)), dtype=torch.int64, device=dev)
                kw = kt = dict(argmax_out=keys, seen=seen, vocab=50257, penalty=1.2)
            res = {}
            splits = (1, 2, 4) if epi == ops.EPI_PARTIAL else (1,)
            for s in splits:
                if (K // s) % 128 or (K // s) * 2 * 64 > 100 * 1024:  # LDS panel must fit
                    continue
                ex = dict(split_k=s) if epi == ops.EPI_PARTIAL else {}
                res[f"ps_s{s}"] = graph_time(lambda i: ops.gemm_ps(a, wsh[i % copies], epi, **kw, **ex))
                if epi == ops.EPI_PARTIAL or s == 1:
                    res[f"tiled_s{s}"] = graph_time(lambda i: ops.gemm(a, ws[i % copies], epi, **kt, **ex))
            for t in forced:
                if epi == ops.EPI_PARTIAL:
                    continue
                L.dlms_gemm_force_tile(t)
                try:
                    res[f"tile{t}"] = graph_time(lambda i: ops.gemm(a, ws[i % copies], epi, **kt))
                finally:
                    L.dlms_gemm_force_tile(-1)
            if epi == ops.EPI_ARGMAX:
                for mt, nt in ((4, 1), (2, 2), (2, 1)):
                    rb = -(-M // (16 * mt))
                    cw = max(1, min(-(-(N // (16 * nt)) // 8), 256 // rb))
                    kk = torch.zeros(M, 8 * cw, dtype=torch.int64, device=dev)
                    kw2 = dict(kw, argmax_out=kk)
                    res[f"ps_{mt}x{nt}"] = graph_time(lambda i: ops.gemm_ps(a, wsh[i % copies], epi, geometry=(mt, nt, cw),
                                                                            **kw2))
            for k, (med, mn) in res.items():
                print(json.dumps({"M": M, "op": op, "variant": k, "us": round(med, 2), "us_min": round(mn, 2),
                                  "TF": round(2 * M * N * K / med / 1e6, 1)}), flush=True)
            del ws, wsh


if __name__ == "__main__":
    main()
