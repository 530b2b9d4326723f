#!/bin/bash
# dataflow decode on GPT-2-medium at batch 1 beside launch-per-op, and an in-kernel trace of the
# GPT-2-124M default geometry (200 CUs, 2 per head)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/df_probe.py --model gpt2-medium --skip-tiny --batch 1 --reps 5 > gpurun_out/dfm.log 2>&1 \
    || { tail -5 gpurun_out/dfm.log; exit 1; }
grep probe gpurun_out/dfm.log | tail -1 | tee gpurun_out/df_medium.jsonl | cut -c1-200
timeout -k 10 200 python -u scripts/df_trace.py --model gpt2 --batch 1 --out gpurun_out/df_trace_g200.json > gpurun_out/dft.log 2>&1 \
    || { tail -5 gpurun_out/dft.log; exit 1; }
tail -3 gpurun_out/dft.log
