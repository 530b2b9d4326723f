#!/bin/bash
# usage: scripts/sweep_bench.sh <tag> "<ENV=..> <ENV=..>" ["..." ...]: one short bench.py run per env set
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/sweep_$tag.jsonl
: > $out
for envs in "$@"; do
  line=$(env $envs timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --latency-batches "" 2>/dev/null | grep '^{') || exit 1
  echo "{\"env\": \"$envs\", \"bench\": $line}" >> $out
  echo "$envs -> $(echo $line | python -c 'import sys,json; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
done
