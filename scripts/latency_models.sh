#!/bin/bash
# single-query latency of every GPT-2 size (bench.py --batch 1), one JSON line each -> gpurun_out/latency_models.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in gpt2 gpt2-medium gpt2-large gpt2-xl; do
    timeout -k 10 300 python -u bench.py --model $m --batch 1 --steps 4 --warmup 1 --latency-batches "" \
        > gpurun_out/lat_$m.log 2>&1 || { tail -5 gpurun_out/lat_$m.log; exit 1; }
    echo "{\"model\": \"$m\", \"bench\": $(grep '^{' gpurun_out/lat_$m.log | tail -1)}" >> gpurun_out/latency_models.jsonl
    tail -1 gpurun_out/latency_models.jsonl | cut -c1-200
done
