#!/bin/bash
# dataflow decode knobs at batch 1 (nt weight stream, grid, attention CUs per head); one JSON line per point
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for envs in "DLMS_DF_NT=0" "DLMS_DF_NT=1" "DLMS_DF_NT=1 DLMS_DF_GRID=128" "DLMS_DF_NT=1 DLMS_DF_GRID=192" "DLMS_DF_NT=1 DLMS_DF_GS=2"; do
    timeout -k 10 150 env $envs python -u scripts/df_probe.py --skip-tiny --no-ref --batch 1 --reps 5 > gpurun_out/df2.log 2>&1 \
        || { tail -5 gpurun_out/df2.log; exit 1; }
    echo "{\"env\": \"$envs\", \"line\": $(grep probe gpurun_out/df2.log | tail -1)}" >> gpurun_out/df_sweep2.jsonl
    tail -1 gpurun_out/df_sweep2.jsonl | cut -c1-160
done
