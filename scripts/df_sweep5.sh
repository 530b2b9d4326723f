#!/bin/bash
# dataflow decode grid around 200 (2 attention CUs per head) at batch 1, repeated points for noise
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # run <ref?> <envs>
    local ref=$1; shift
    timeout -k 10 200 env "$@" python -u scripts/df_probe.py --skip-tiny $ref --batch 1 --reps 7 > gpurun_out/df5.log 2>&1 \
        || { tail -5 gpurun_out/df5.log; exit 1; }
    echo "{\"env\": \"$*\", \"line\": $(grep probe gpurun_out/df5.log | tail -1)}" >> gpurun_out/df_sweep5.jsonl
    python -c "import json; d=json.loads(open('gpurun_out/df_sweep5.jsonl').readlines()[-1]); print(d['env'], d['line']['df_p50_ms'], d['line'].get('ref_p50_ms'))"
}
run "" DLMS_DF_GRID=200 DLMS_DF_GS=2
for g in 196 204 208 216 200 192; do run --no-ref DLMS_DF_GRID=$g DLMS_DF_GS=2; done
