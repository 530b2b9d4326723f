#!/bin/bash
# GPU tests (full -m gpu tier) + gate-under-concurrency bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
timeout -k 10 700 $T -m gpu tests/ > gpurun_out/r2_g_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2_g_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_gate.py --clients 100 --rounds 5 > gpurun_out/r2_gate_echo.log 2>&1 || exit $?
cat gpurun_out/r2_gate_echo.log | grep gate_concurrency
timeout -k 10 300 python -u scripts/bench_gate.py --clients 100 --rounds 3 --tutor gpt2 > gpurun_out/r2_gate_gpt2.log 2>&1 || exit $?
cat gpurun_out/r2_gate_gpt2.log | grep gate_concurrency
