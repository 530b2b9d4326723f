#!/bin/bash
# Latency path: kernel + engine numerics, TP functional test, then a B=1 kernel profile.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_skinny_gpu.py tests/test_engine_gpu.py tests/test_tp_gpu.py > gpurun_out/r2_lat_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_lat_tests.log
[ $rc -ge 2 ] && exit $rc
bash scripts/prof_bench.sh b1_v2 --batch 1 --steps 3 --warmup 1 --latency-batches ""
