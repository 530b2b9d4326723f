#!/bin/bash
# fp8 (W8A8 e4m3 QKV / c_fc / LM head, bf16 latency path) vs bf16 on GPT-2-XL, one MI355X (VERDICT r5
# next #3): decode at 64 / 256 / 512 rows and the packed prefill.  -> gpurun_out/fp8_ab.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 512 256 64; do
    for dt in bf16 fp8; do
        timeout -k 10 400 python -u bench.py --model gpt2-xl --batch $b --steps 3 --warmup 1 --weight-dtype $dt \
            --latency-batches "" > gpurun_out/fp8_ab_run.log 2>&1 || { tail -5 gpurun_out/fp8_ab_run.log; exit 1; }
        echo "{\"batch\": $b, \"weight_dtype\": \"$dt\", \"bench\": $(grep '^{' gpurun_out/fp8_ab_run.log | tail -1)}" \
            >> gpurun_out/fp8_ab.jsonl
        tail -1 gpurun_out/fp8_ab.jsonl | cut -c1-200
    done
done
