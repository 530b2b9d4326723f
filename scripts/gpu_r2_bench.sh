#!/bin/bash
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_skinny_gpu.py tests/test_engine_gpu.py > gpurun_out/r2_b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_b_tests.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2_b_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2_b_bench.log
