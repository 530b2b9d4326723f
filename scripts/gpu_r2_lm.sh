#!/bin/bash
# Batch-1 LM head A/B: tiled vs skinny, nt vs default weight loads.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_skinny_gpu.py -k "argmax" > gpurun_out/r2_lm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2_lm_tests.log
[ $rc -ne 0 ] && exit $rc
for v in "0 1" "1 0" "1 1"; do
  set -- $v
  DLMS_LM_SKINNY=$1 DLMS_LM_NT=$2 timeout -k 10 200 python -u bench.py --batch 1 --steps 5 --warmup 2 --latency-batches "" > gpurun_out/r2_lm_$1$2.log 2>&1 || exit $?
  echo "skinny=$1 nt=$2 $(grep -o '"p50_query_latency_ms": [0-9.]*' gpurun_out/r2_lm_$1$2.log)"
done
