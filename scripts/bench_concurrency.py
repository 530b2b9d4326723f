#!/usr/bin/env python3
"""Do independent small kernels on different HIP streams run side by side?  Times N launches of a
latency-bound kernel (skinny QKV at 8 rows, ~150 workgroups) on one stream, then the same N on each
of k streams at once -- eager launches and hipGraph replays -- and reports the concurrency factor
(k * t_one / t_k; k = perfect overlap, 1 = serialised)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_lms_raft_llm_amd import ops  # noqa: E402


def main():
    ops.lib()
    dev = "cuda"
    M, K, N, n = 8, 768, 2304, 200
    streams = [torch.cuda.Stream() for _ in range(4)]
    bufs = []
    for _ in range(4):
        x = torch.randn(M, K, device=dev)
        w = ops.shuffle_weight((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16))
        g, b = torch.ones(K, device=dev), torch.zeros(K, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bufs.append((x, w, g, b, out))

    def work(i, reps):
        x, w, g, b, out = bufs[i]
        for _ in range(reps):
            ops.skinny_gemm(x, w, ops.EPI_BF16, ln=(g, b, 1e-5), out=out)

    def timed(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    # eager
    for k in (1, 2, 4):
        def run(k=k):
            for i in range(k):
                with torch.cuda.stream(streams[i]):
                    work(i, n)
        run()
        t = min(timed(run) for _ in range(3))
        print(json.dumps({"mode": "eager", "streams": k, "ms": round(t, 3), "us_per_kernel": round(t * 1e3 / (n * k), 2)}),
              flush=True)
    # graphs: one graph per stream, replayed concurrently
    graphs = []
    for i in range(4):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(streams[i]):
            work(i, 2)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            work(i, n)
        graphs.append(g)
    for k in (1, 2, 4):
        def run(k=k):
            for i in range(k):
                with torch.cuda.stream(streams[i]):
                    graphs[i].replay()
        run()
        t = min(timed(run) for _ in range(3))
        print(json.dumps({"mode": "graph", "streams": k, "ms": round(t, 3), "us_per_kernel": round(t * 1e3 / (n * k), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
