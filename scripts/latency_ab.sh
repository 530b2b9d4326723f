#!/bin/bash
# batch-1 latency A/B for one model: latency_ab.sh <model> "<ENV=v,...>;<ENV=v,...>;..."  -> gpurun_out/latency_ab.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
m=$1
IFS=';' read -ra sets <<< "$2"
for envs in "${sets[@]}"; do
    timeout -k 10 300 env ${envs//,/ } python -u bench.py --model $m --batch 1 --steps 4 --warmup 1 --latency-batches "" \
        > gpurun_out/lat_ab.log 2>&1 || { tail -5 gpurun_out/lat_ab.log; exit 1; }
    echo "{\"model\": \"$m\", \"env\": \"$envs\", \"bench\": $(grep '^{' gpurun_out/lat_ab.log | tail -1)}" >> gpurun_out/latency_ab.jsonl
    python -c "import json,sys; d=json.loads(open('gpurun_out/latency_ab.jsonl').readlines()[-1]); print(d['model'], d['env'], d['bench']['p50_query_latency_ms'])"
done
