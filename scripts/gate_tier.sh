#!/bin/bash
# The relevance gate as one GPU-tier service: the LMS path with GPU-less LMS
# nodes calling ONE gate server (--gate remote: hosted by the tutor; remote-proc: its own process)
# against the Tutoring path, one query at a time and at the saturating 5.5 k q/s.
#   gpurun -- bash scripts/gate_tier.sh [which ...]     -> gpurun_out/gate_tier.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/gate_tier.jsonl
run() {  # run <tag> <bench_grpc args...>
    local tag=$1
    shift
    timeout -k 10 300 python -u scripts/bench_grpc.py "$@" --out $O --log gpurun_out/gate_tier_$tag.log --tag $tag \
        > gpurun_out/gate_tier_$tag.out 2>&1 || { tail -20 gpurun_out/gate_tier_$tag.out; exit 1; }
    tail -1 gpurun_out/gate_tier_$tag.out | cut -c1-600
}
for w in ${@:-closed open}; do
    case $w in
        closed)
            run closed1_tutoring --target tutoring --closed 1 --duration 15 --warmup 6 --frontends 2
            run closed1_lms_remote --target lms --gate remote --closed 1 --duration 15 --warmup 6 --frontends 2 ;;
        open)
            run open5500_tutoring --target tutoring --rates 5500 --duration 20 --warmup 8 --client-procs 8
            run open5500_lms_remote --target lms --gate remote --rates 5500 --duration 20 --warmup 8 --client-procs 8 ;;
        openproccu)  # the gate server's passes under load on 16 / 32 CUs
            DLMS_GATE_CUS=16 run open5500_lms_remote_proc_cu16 --target lms --gate remote-proc --rates 5500 \
                --duration 20 --warmup 8 --client-procs 8
            DLMS_GATE_CUS=32 run open5500_lms_remote_proc_cu32 --target lms --gate remote-proc --rates 5500 \
                --duration 20 --warmup 8 --client-procs 8 ;;
        opennogate)  # the LMS path without any gate: what the LMS tier itself costs on this box
            run open5500_lms_nogate --target lms --gate off --rates 5500 --duration 20 --warmup 8 --client-procs 8 ;;
        openproc)
            run open5500_lms_remote_proc --target lms --gate remote-proc --rates 5500 --duration 20 --warmup 8 \
                --client-procs 8 ;;
    esac
done
