#!/bin/bash
# Dataflow-decode A/B sweep (replaces the round-3 one-off df_sweep2..5 / df_medium / df_loader_ab
# scripts): one scripts/df_probe.py run per point, one JSON line per point.
#
#   bash scripts/df_sweep.sh [-m MODEL] [-b BATCHES] [-r REPS] [-o OUT.jsonl] [--ref] POINT [POINT ...]
#
# POINT: a comma-separated env set ("DLMS_DF_GRID=192,DLMS_DF_GS=2"), "default", or
#        "lib=<file in ops/_lib>[,ENV=v...]" for a library variant built with
#        ops.build(out=..., defines=...) (loaded through DLMS_HIP_LIB).
# --ref: also time the launch-per-op path at every point (df_probe without --no-ref).
# Every run has its own time limit; the first failing run ends the sweep (no GPU work after it).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
model=gpt2 batches=1 reps=5 out=gpurun_out/df_sweep.jsonl ref=--no-ref
while [ $# -gt 0 ]; do
    case "$1" in
        -m) model=$2; shift 2 ;;
        -b) batches=$2; shift 2 ;;
        -r) reps=$2; shift 2 ;;
        -o) out=$2; shift 2 ;;
        --ref) ref=""; shift ;;
        *) break ;;
    esac
done
L=distributed_lms_raft_llm_amd/ops/_lib
for point in "$@"; do
    envs=()
    IFS=',' read -ra items <<< "$point"
    for it in "${items[@]}"; do
        case "$it" in
            default) ;;
            lib=*) envs+=("DLMS_HIP_LIB=$L/${it#lib=}") ;;
            *) envs+=("$it") ;;
        esac
    done
    for b in ${batches//,/ }; do
        timeout -k 10 300 env "${envs[@]}" python -u scripts/df_probe.py --model "$model" --skip-tiny $ref --batch "$b" \
            --reps "$reps" > gpurun_out/df_sweep.log 2>&1 || { tail -5 gpurun_out/df_sweep.log; exit 1; }
        echo "{\"point\": \"$point\", \"model\": \"$model\", \"batch\": $b, \"line\": $(grep probe gpurun_out/df_sweep.log | tail -1)}" >> "$out"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); l=d['line']; print(d['point'], d['batch'], l['df_p50_ms'], l.get('ref_p50_ms'))" "$out"
    done
done
