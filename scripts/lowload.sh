#!/bin/bash
# One query at a time through gRPC: the reference's own operating point
# (lms_server.py:1237-1274 -> tutoring_server.py:15-31).  LMS.GetLLMAnswer on a 3-node Raft cluster
# whose BERT gates share the tutor's GPU, and Tutoring.GetLLMAnswer direct, closed loop with one client.
#   gpurun -- bash scripts/lowload.sh [duration_s]   -> gpurun_out/lowload.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
D=${1:-20}
for tgt in tutoring lms; do
    timeout -k 10 420 python -u scripts/bench_grpc.py --target $tgt --closed 1 --duration $D --warmup 8 \
        --frontends 2 --out gpurun_out/lowload.jsonl --log gpurun_out/lowload_$tgt.log --tag closed1 \
        > gpurun_out/lowload_$tgt.out 2>&1 || { tail -20 gpurun_out/lowload_$tgt.out; exit 1; }
    tail -1 gpurun_out/lowload_$tgt.out | cut -c1-700
done
