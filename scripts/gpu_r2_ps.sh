#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_skinny_gpu.py -k "gemm_ps" > gpurun_out/r2_ps_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2_ps_tests.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_ps.py --ops lmhead --batches 256,512,1024 > gpurun_out/r2_ps_bench3.log 2>&1
