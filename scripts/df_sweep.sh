#!/bin/bash
# dataflow decode A/B: residual copies (library variants) x grid size; one JSON line per point
set -o pipefail
for c in 2 4 8; do
  for g in 256 128; do
    DLMS_HIP_LIB=distributed_lms_raft_llm_amd/ops/_lib/libdlms_hip_c$c.so DLMS_DF_GRID=$g \
      timeout -k 10 120 python -u scripts/df_probe.py --skip-tiny --no-ref --batch 1 --reps 5 > gpurun_out/df_sweep_c${c}_g${g}.log 2>&1 || exit 1
    echo "{\"copies\": $c, \"grid\": $g, \"line\": $(grep probe gpurun_out/df_sweep_c${c}_g${g}.log)}" >> gpurun_out/df_sweep.jsonl
  done
done
