#!/bin/bash
# dataflow decode grid x attention-CUs-per-head x weight-stream policy at batch 1, beside the
# launch-per-op path on the same box; one JSON line per point -> gpurun_out/df_sweep3.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/df_probe.py --skip-tiny --batch 1 --reps 5 > gpurun_out/df3.log 2>&1 || { tail -5 gpurun_out/df3.log; exit 1; }
echo "{\"env\": \"default (with launch-per-op ref)\", \"line\": $(grep probe gpurun_out/df3.log | tail -1)}" >> gpurun_out/df_sweep3.jsonl
for envs in "DLMS_DF_GRID=192" "DLMS_DF_NT=1 DLMS_DF_GRID=192 DLMS_DF_GS=2" "DLMS_DF_GRID=192 DLMS_DF_GS=2" \
            "DLMS_DF_NT=1 DLMS_DF_GRID=160" "DLMS_DF_NT=1 DLMS_DF_GRID=176" "DLMS_DF_NT=1 DLMS_DF_GRID=208" \
            "DLMS_DF_NT=1 DLMS_DF_GRID=224" "DLMS_DF_NT=1 DLMS_DF_GRID=192"; do
    timeout -k 10 150 env $envs python -u scripts/df_probe.py --skip-tiny --no-ref --batch 1 --reps 5 > gpurun_out/df3.log 2>&1 \
        || { tail -5 gpurun_out/df3.log; exit 1; }
    echo "{\"env\": \"$envs\", \"line\": $(grep probe gpurun_out/df3.log | tail -1)}" >> gpurun_out/df_sweep3.jsonl
    python -c "import json; d=json.loads(open('gpurun_out/df_sweep3.jsonl').readlines()[-1]); print(d['env'], d['line']['df_p50_ms'])"
done
