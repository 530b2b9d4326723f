#!/bin/bash
# Default bench (headline + B=1/B=32 latency keys), B=1024 kernel profile, B=8 T=1024 attention bench.
set -e
cd "$GRAFT_REPO_ROOT"
S=scripts/gpu_step.sh
L=gpurun_out/r2_prof.log
$S 400 $L python -u bench.py
tail -1 $L
bash scripts/prof_bench.sh b1024 --steps 5 --warmup 2 --latency-batches ""
$S 300 $L python -u scripts/bench_skinny.py --batches 8 --T 1024
grep attn_T1024 $L
