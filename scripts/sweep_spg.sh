#!/bin/bash
# decode steps per graph replay on the mid path (DLMS_STEPS_PER_GRAPH_SMALL) at 8 / 16 / 32 / 64 rows
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 4 8 16; do
    timeout -k 10 300 env DLMS_STEPS_PER_GRAPH_SMALL=$v python -u bench.py --batch 64 --steps 3 --warmup 1 \
        --latency-batches 8,16,32 > gpurun_out/spg.log 2>&1 || exit 1
    echo "{\"steps_per_graph_small\": $v, \"bench\": $(grep '^{' gpurun_out/spg.log | tail -1)}" >> gpurun_out/spg.jsonl
done
