#!/bin/bash
# Round-2 baseline: latency (B=1, B=32) and headline (B=1024) bench + kernel stats at B=1.
set -e
cd "$GRAFT_REPO_ROOT"
S=scripts/gpu_step.sh
L=gpurun_out/r2_baseline.log
$S 300 $L python bench.py --batch 1 --steps 5 --warmup 2
$S 300 $L python bench.py --batch 32 --steps 5 --warmup 2
$S 300 $L python bench.py --steps 10 --warmup 3
bash scripts/prof_bench.sh b1 --batch 1 --steps 3 --warmup 1
