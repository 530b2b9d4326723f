#!/bin/bash
# Batch-1 latency sweep: one bench.py run per (env setting, model); each run under its own time
# limit, the first failure ends the sweep.  Usage:
#   bash scripts/sweep_latency.sh <out.jsonl> "<ENV=v,...>;<ENV=v,...>" "gpt2 gpt2-medium" [batch]
set -u
out=$1; envsets=$2; models=$3; batch=${4:-1}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IFS=';' read -ra sets <<< "$envsets"
for envs in "${sets[@]}"; do
    for m in $models; do
        line=$(timeout -k 10 300 env ${envs//,/ } python -u bench.py --model "$m" --batch "$batch" --steps 5 --warmup 2 \
               --latency-batches "" 2>>gpurun_out/sweep_latency.err | grep '^{' | tail -1)
        rc=$?
        if [ $rc -ne 0 ] || [ -z "$line" ]; then echo "run failed: $envs $m rc=$rc" >&2; exit 1; fi
        echo "{\"env\": \"$envs\", \"model\": \"$m\", \"batch\": $batch, \"bench\": $line}" >> "$out"
        python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], sys.argv[3], d['p50_query_latency_ms'])" "$line" "$envs" "$m"
    done
done
