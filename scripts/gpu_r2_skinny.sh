#!/bin/bash
# Latency-path kernels: numerics tests, then the microbench.
cd "$GRAFT_REPO_ROOT"
L=gpurun_out/r2_skinny.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_skinny_gpu.py > gpurun_out/r2_skinny_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2_skinny_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/bench_skinny.py > $L 2>&1
