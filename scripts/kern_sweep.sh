#!/bin/bash
# decode-GEMM tile sweep at the overlapped step's row halves (M 512) and the full batch
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_kernels.py --batches 512,1024 --tiles=-1,1,4,17,18,19 \
    --ops qkv,oproj,fc,proj > gpurun_out/kern_sweep.jsonl 2>&1
