#!/bin/bash
# dataflow decode around grid 192 / 2 attention CUs per head at batch 1, then batch 2 beside the
# launch-per-op path; one JSON line per point -> gpurun_out/df_sweep4.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # run <batch> <ref?> <envs>
    local b=$1 ref=$2; shift 2
    timeout -k 10 200 env "$@" python -u scripts/df_probe.py --skip-tiny $ref --batch $b --reps 5 > gpurun_out/df4.log 2>&1 \
        || { tail -5 gpurun_out/df4.log; exit 1; }
    echo "{\"env\": \"$*\", \"line\": $(grep probe gpurun_out/df4.log | tail -1)}" >> gpurun_out/df_sweep4.jsonl
    python -c "import json; d=json.loads(open('gpurun_out/df_sweep4.jsonl').readlines()[-1]); print(d['env'], d['line']['B'], d['line']['df_p50_ms'], d['line'].get('ref_p50_ms'))"
}
run 1 "" DLMS_DF_GRID=192 DLMS_DF_GS=2
run 1 --no-ref DLMS_DF_GRID=192 DLMS_DF_GS=1
run 1 --no-ref DLMS_DF_GRID=184 DLMS_DF_GS=2
run 1 --no-ref DLMS_DF_GRID=200 DLMS_DF_GS=2
run 1 --no-ref DLMS_DF_GRID=168 DLMS_DF_GS=2
run 2 "" DLMS_DF_GRID=192 DLMS_DF_GS=2
run 2 --no-ref DLMS_DF_GRID=192 DLMS_DF_GS=4
