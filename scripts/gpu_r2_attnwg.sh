#!/bin/bash
# Cross-workgroup split attention: numerics, then the sync-mode x B sweep at T=1024.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_skinny_gpu.py -k "attention" > gpurun_out/r2_awg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_awg_tests.log
[ $rc -ne 0 ] && exit $rc
for m in 0 1 2; do
  DLMS_ATTN_SPLIT_SYNC=$m timeout -k 10 200 python -u scripts/bench_skinny.py --attn-only --batches 1,8,32 --T 1024 > gpurun_out/r2_awg_bench$m.log 2>&1 || exit $?
  echo "sync=$m"; grep splitwg gpurun_out/r2_awg_bench$m.log
done
