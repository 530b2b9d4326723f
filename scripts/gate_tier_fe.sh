#!/bin/bash
# Tutor-served gate (--serve-gate) at 5.5 k q/s: front-end count and the least gap between gate
# passes, against gate_tier.sh's default (4 front ends, 10 ms).   -> gpurun_out/gate_tier_fe.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/gate_tier_fe.jsonl
run() {
    local tag=$1
    shift
    timeout -k 10 300 python -u scripts/bench_grpc.py "$@" --out $O --log gpurun_out/gate_tier_fe_$tag.log --tag $tag \
        > gpurun_out/gate_tier_fe_$tag.out 2>&1 || { tail -20 gpurun_out/gate_tier_fe_$tag.out; exit 1; }
    tail -1 gpurun_out/gate_tier_fe_$tag.out | cut -c1-400
}
run open5500_lms_remote_fe8 --target lms --gate remote --rates 5500 --duration 20 --warmup 8 --client-procs 8 --frontends 8
DLMS_GATE_MIN_GAP_MS=2 run open5500_lms_remote_gap2 --target lms --gate remote --rates 5500 --duration 20 --warmup 8 --client-procs 8
