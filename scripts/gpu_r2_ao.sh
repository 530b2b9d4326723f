#!/bin/bash
# Fused attention + out-projection: kernel numerics, engine/TP oracles, then batch-1/4 latency A/B.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 180 --timeout-method thread"
timeout -k 10 300 $T tests/test_skinny_gpu.py -k "oproj or attention_split or many_slabs" > gpurun_out/r2_ao_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2_ao_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 $T tests/test_engine_gpu.py tests/test_tp_gpu.py > gpurun_out/r2_ao_tests2.log 2>&1
rc=$?; tail -2 gpurun_out/r2_ao_tests2.log
[ $rc -ne 0 ] && exit $rc
for f in 1 0; do
  DLMS_FUSE_ATTN_OPROJ=$f timeout -k 10 200 python -u bench.py --batch 4 --steps 3 --warmup 1 --latency-batches 1 > gpurun_out/r2_ao_$f.log 2>&1 || exit $?
  echo "fuse=$f $(grep -o '"p50_query_latency_ms[_b1]*": [0-9.]*' gpurun_out/r2_ao_$f.log | tr '\n' ' ')"
done
