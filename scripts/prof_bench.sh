#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench.py run; summary CSV -> gpurun_out/prof_<tag>/
set -e
tag=${1:-bench}; shift || true
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/prof_$tag/bench.log 2>&1
find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_$tag/kernel_stats.csv
rm -f gpurun_out/prof_$tag/run_kernel_trace.csv
find gpurun_out/prof_$tag -name "*_kernel_trace.csv" -delete
tail -1 gpurun_out/prof_$tag/bench.log
