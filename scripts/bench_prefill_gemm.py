#!/usr/bin/env python3
"""Packed-prefill GEMMs (1024 prompts x 32 tokens = 32768 rows, GPT-2-124M shapes): our MFMA GEMM
with its fused epilogue vs hipBLASLt (torch.mm, plain bf16 out) -- how far the big-M path is from
the library and from the MFMA peak.  JSON lines: op, variant, us, TFLOP/s."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_lms_raft_llm_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--tiles", default="", help="comma list of forced tile ids (dlms_gemm_force_tile) to time too")
    ap.add_argument("--ops", default="qkv,oproj,fc,proj")
    args = ap.parse_args()
    L = ops.lib()
    forced = [int(t) for t in args.tiles.split(",") if t.strip()]
    M, D = args.M, args.d
    dev = "cuda"
    shapes = {"qkv": (3 * D, D, ops.EPI_BF16), "oproj": (D, D, ops.EPI_PARTIAL), "fc": (4 * D, D, ops.EPI_GELU_TANH),
              "proj": (D, 4 * D, ops.EPI_PARTIAL)}
    for op, (N, K, epi) in shapes.items():
        if op not in args.ops.split(","):
            continue
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        flop = 2.0 * M * N * K
        res = {}
        if epi == ops.EPI_PARTIAL:
            for split in (1, 2):
                parts = torch.empty(split, M, N, device=dev)
                res[f"ours_partial_s{split}"] = timed(lambda: ops.gemm(a, w, epi, out=parts, split_k=split))
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            res["ours_" + ("gelu" if epi == ops.EPI_GELU_TANH else "bf16")] = timed(
                lambda: ops.gemm(a, w, epi, bias=bias, out=out))
        o2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res["hipblaslt_bf16"] = timed(lambda: torch.mm(a, w.t(), out=o2))
        ref = torch.mm(a.float(), w.float().t())
        errs = {}
        # forced tile configs (plain bf16 epilogue for the column-parallel ops, split-K 1 partials
        # for the row-parallel ones), each checked against the fp32 product
        for t in forced:
            L.dlms_gemm_force_tile(t)
            try:
                if epi == ops.EPI_PARTIAL:
                    parts = torch.empty(1, M, N, device=dev)
                    fn = lambda: ops.gemm(a, w, epi, out=parts, split_k=1)  # noqa: E731
                    fn()
                    got = parts[0]
                else:
                    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                    fn = lambda: ops.gemm(a, w, ops.EPI_BF16, bias=bias, out=out)  # noqa: E731
                    fn()
                    got = out.float()
                torch.cuda.synchronize()
                errs[f"tile{t}"] = float(((got - ref).abs().max() / ref.abs().max()).item())
                res[f"tile{t}"] = timed(fn)
            finally:
                L.dlms_gemm_force_tile(-1)
        for k, us in res.items():
            print(json.dumps({"M": M, "op": op, "N": N, "K": K, "variant": k, "us": round(us, 1),
                              "TFLOPs": round(flop / us / 1e6, 1), "max_rel_err": errs.get(k)}), flush=True)


if __name__ == "__main__":
    main()
