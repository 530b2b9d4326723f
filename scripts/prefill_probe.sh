#!/bin/bash
# batch-1 prefill probe after a 1024-query run (bench.py order), A/B against launch-per-op and a short bench line
#   gpurun -- bash scripts/prefill_probe.sh   -> gpurun_out/prefill_probe.jsonl, gpurun_out/bench_probe.log
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
o=gpurun_out/prefill_probe.jsonl
timeout -k 10 200 python -u scripts/prefill_probe.py --warm-batch 1024 >> $o 2>gpurun_out/pp.err && \
timeout -k 10 200 env DLMS_DATAFLOW=0 python -u scripts/prefill_probe.py --warm-batch 1024 >> $o 2>>gpurun_out/pp.err && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 >> gpurun_out/bench_probe.log 2>&1
cat $o; grep '^{' gpurun_out/bench_probe.log
