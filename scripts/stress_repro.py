"""Repro for the open stress issue (docs/PERFORMANCE.md, tests/test_dataflow_gpu.py::
test_dataflow_beside_a_long_kernel_on_another_stream): after a pooled torch stream ran GEMMs (and a
dataflow decode ran beside them), a later engine's graph replay segfaulted.

    python scripts/stress_repro.py <mode>
      gemm      : 80 x 8192^3 torch.mm on a pooled side stream, then the test-46 engine (graphs, 10 rows)
      gemm_df   : the same with a batch-1 dataflow generate beside the GEMMs (the stress test)
      df        : the dataflow generate alone, then the test-46 engine
      none      : the test-46 engine only
      gemm_cap  : the GEMMs on torch's default graph-capture stream (the pooled stream every
                  torch.cuda.graph capture uses), then the test-46 engine
"""
import os
import sys

import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(mode: str):
    from test_engine_gpu import _prompts, _setup

    from distributed_lms_raft_llm_amd.engine.gpt2_engine import HipGPT2Engine

    cfg, w = _setup("gpt2")
    if mode == "gemm_cap":
        g0 = torch.cuda.CUDAGraph()  # creates torch.cuda.graph.default_capture_stream
        x = torch.zeros(4, device="cuda")
        with torch.cuda.graph(g0):
            x += 1
        cap = torch.cuda.graph.default_capture_stream
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        c = torch.empty_like(a)
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            for _ in range(80):
                torch.mm(a, a, out=c)
        cap.synchronize()
        print("gemms on the capture stream done", flush=True)
    if mode in ("gemm", "gemm_df", "df"):
        eng = HipGPT2Engine(cfg, w, max_batch=2, max_length=150) if mode != "gemm" else None
        p1 = _prompts(cfg, [32], seed=5)
        if eng is not None:
            eng.generate(p1)
        side = torch.cuda.Stream()
        if mode != "df":
            a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
            c = torch.empty_like(a)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(80):
                    torch.mm(a, a, out=c)
        if eng is not None:
            eng.generate(p1)
            print("df aborts", eng.df_aborts, flush=True)
        side.synchronize()
        del eng
    print("stage 1 done", flush=True)
    prompts = _prompts(cfg, [32] * 6 + [9, 17, 3, 25], seed=5)
    for parts in (2, 4):
        ov = HipGPT2Engine(cfg, w, max_batch=16, max_length=72, use_graph=True, overlap=True, overlap_min_batch=2,
                           overlap_parts=parts)
        a1 = ov.generate(prompts)
        print("parts", parts, "ok", len(a1), flush=True)
    print("REPRO PASSED", mode, flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
