#!/bin/bash
# dataflow decode loader variants (in-flight depth, loader waves) at batch 1, interleaved A/B:
# one JSON line per point -> gpurun_out/df_loader_ab.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=distributed_lms_raft_llm_amd/ops/_lib
for lib in libdlms_hip.so libdlms_hip_infl64.so libdlms_hip_nl3.so libdlms_hip_nl3i64.so libdlms_hip.so libdlms_hip_nl3i64.so; do
    timeout -k 10 150 env DLMS_HIP_LIB=$L/$lib python -u scripts/df_probe.py --skip-tiny --no-ref --batch 1 --reps 7 \
        > gpurun_out/dfl.log 2>&1 || { tail -5 gpurun_out/dfl.log; exit 1; }
    echo "{\"lib\": \"$lib\", \"line\": $(grep probe gpurun_out/dfl.log | tail -1)}" >> gpurun_out/df_loader_ab.jsonl
    python -c "import json; d=json.loads(open('gpurun_out/df_loader_ab.jsonl').readlines()[-1]); print(d['lib'], d['line']['df_p50_ms'], d['line']['df_tokens'][:6])"
done
