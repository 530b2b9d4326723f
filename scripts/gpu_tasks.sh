#!/bin/bash
# One entry point for the GPU-box work of this repo (replaces the per-experiment lease scripts):
#
#   gpurun -- bash scripts/gpu_tasks.sh <task> [<task> ...]
#
# tasks (run in order; the first failing step ends the call -- no GPU work after a fault/timeout):
#   tests            full `pytest -m gpu` tier                     -> gpurun_out/tests.log
#   test:<path>      one test file / node id of the gpu tier       -> gpurun_out/test_sel.log
#   smoke            __graft_entry__.smoke()
#   bench            default bench.py (headline + b1/b32 keys)    -> gpurun_out/bench.log
#   prof:<tag>       rocprofv3 kernel stats of a short bench.py run (B=1024)   -> gpurun_out/prof_<tag>/
#   prof1:<tag>      the same at batch 1
#   profm:<tag>:<model>:<batch>  the same for another model / batch
#   pmc:<tag>:<batch>  three rocprofv3 --pmc passes (SQ / TCC fetch / TCC write) of an eager bench.py run
#                    -> gpurun_out/pmc_<tag>/summary.json
#   trace:<tag>      per-dispatch kernel trace of one B=1024 generation (timeline analysis) -> gpurun_out/trace_<tag>/
#   skinny           latency-path kernel microbench                -> gpurun_out/skinny.jsonl
#   attn             split-K flash-decode sweep (B x T x waves x workgroups)   -> gpurun_out/attn.jsonl
#   pgemm            packed-prefill GEMMs (32768 rows) vs hipBLASLt -> gpurun_out/pgemm.jsonl
#   pgemmt:<ids>     the same plus forced tile configs (dlms_gemm_force_tile ids, ',')
#   ps               panel-resident LM-head GEMM vs tiled          -> gpurun_out/ps.jsonl
#   pst:<ids>        LM head at 512 rows, gemm_ps vs forced tiled configs
#   gate             relevance gate under 100 concurrent GetLLMAnswer calls    -> gpurun_out/gate.jsonl
#   serving          open-loop Poisson serving at 20 / 200 / 1000 queries/s      -> gpurun_out/serving.jsonl
#   grpc:<tgt>:<rates>[:<ENV=v,..>] scripts/bench_grpc.py --target tutoring|lms at those offered q/s -> gpurun_out/grpc.jsonl
#   e2e:<n>          scripts/run_config.py --config n (Raft cluster + gate + tutor) -> gpurun_out/e2e_<n>.log
#   e2e1:<n>         the same with the tutor at TP=1 (one-GPU boxes: configs 4/5 ask for TP=4/8)
#   sweep:<ENV=v,..> one bench.py run per ';'-separated env set   -> gpurun_out/sweep.jsonl
#   sweep1:<...>     the same at batch 1 and 2 (p50 per query)     -> gpurun_out/sweep1.jsonl
#   sweep4:<...>     the same at batch 3 and 4
#   sweep32:<...>    the same at batch 16 and 32                   -> gpurun_out/sweep1.jsonl
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 180 --timeout-method thread"

step() {  # step <seconds> <log> <cmd...>: own time limit; a fault, abort or timeout ends the call
    local secs=$1 log=$2
    shift 2
    echo "=== $(date +%T) $*" >> "$log"
    timeout -k 10 "$secs" "$@" >> "$log" 2>&1
    local rc=$?
    echo "=== rc=$rc" >> "$log"
    [ $rc -ne 0 ] && { echo "step failed rc=$rc: $*" >&2; tail -5 "$log" >&2; exit $rc; }
    return 0
}

prof() {  # prof <tag> <bench args...>
    local tag=$1
    shift
    export TMPDIR=/tmp
    mkdir -p gpurun_out/prof_$tag
    step 300 gpurun_out/prof_$tag/bench.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run \
        --output-format csv -- python3 bench.py "$@"
    find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_$tag/kernel_stats.csv
    find gpurun_out/prof_$tag -name "*_kernel_trace.csv" -delete
    python scripts/kstats.py gpurun_out/prof_$tag/kernel_stats.csv > gpurun_out/prof_$tag/summary.txt
    head -12 gpurun_out/prof_$tag/summary.txt
}

for task in "$@"; do
    case "$task" in
        tests) step 900 gpurun_out/tests.log $T -m gpu tests/; tail -2 gpurun_out/tests.log ;;
        testall:*)  # the same without -x: every failure of the selection is reported (the call still ends on it)
            step 900 gpurun_out/test_all.log python -u -m pytest -q -rf --timeout 180 --timeout-method thread -m gpu \
                ${task#testall:}; tail -2 gpurun_out/test_all.log ;;
        test:*) step 600 gpurun_out/test_sel.log $T -m gpu ${task#test:}; tail -2 gpurun_out/test_sel.log ;;
        testenv:*)  # testenv:<ENV=v>:<paths>  one gpu test selection under an environment setting
            spec=${task#testenv:}; envs=${spec%%:*}; paths=${spec#*:}
            step 600 gpurun_out/test_env.log env ${envs//,/ } $T -m gpu $paths; tail -2 gpurun_out/test_env.log ;;
        smoke) step 300 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()"; tail -2 gpurun_out/smoke.log ;;
        bench) step 600 gpurun_out/bench.log python -u bench.py; grep '^{' gpurun_out/bench.log | tail -1 ;;
        benchng) step 600 gpurun_out/bench_ng.log python -u bench.py --no-graph --latency-batches 32
                 grep '^{' gpurun_out/bench_ng.log | tail -1 ;;
        prof:*) prof "${task#prof:}" --steps 5 --warmup 2 --latency-batches "" ;;
        prof1:*) prof "${task#prof1:}" --batch 1 --steps 3 --warmup 1 --latency-batches "" ;;
        prof32:*) prof "${task#prof32:}" --batch 32 --steps 3 --warmup 1 --latency-batches "" ;;
        profm:*)  # profm:<tag>:<model>:<batch>
            spec=${task#profm:}; tag=${spec%%:*}; rest=${spec#*:}; model=${rest%%:*}; batch=${rest#*:}
            prof "$tag" --model "$model" --batch "$batch" --steps 3 --warmup 1 --latency-batches "" ;;
        pmc:*)
            spec=${task#pmc:}; tag=${spec%%:*}; batch=${spec#*:}; export TMPDIR=/tmp; D=gpurun_out/pmc_$tag; mkdir -p $D
            passes=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
                    "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum")
            i=0
            for ctrs in "${passes[@]}"; do
                i=$((i + 1))
                step 240 $D/pass$i.log timeout -s KILL 200 rocprofv3 --pmc $ctrs -d $D/p$i -o run --output-format csv \
                    -- python3 bench.py --batch $batch --steps 1 --warmup 0 --no-graph --latency-batches ""
            done
            step 120 $D/summary.txt python scripts/pmc_summary.py $D/summary.json $(find $D -name "*counter_collection.csv")
            find $D -name "*counter_collection.csv" -delete
            cat $D/summary.txt ;;
        trace:*)
            tag=${task#trace:}; export TMPDIR=/tmp; mkdir -p gpurun_out/trace_$tag
            step 300 gpurun_out/trace_$tag/bench.log rocprofv3 --kernel-trace -d gpurun_out/trace_$tag -o run \
                --output-format csv -- python3 bench.py --steps 1 --warmup 1 --latency-batches ""
            f=$(find gpurun_out/trace_$tag -name "*kernel_trace.csv" | head -1)
            step 120 gpurun_out/trace_$tag/timeline.txt python scripts/timeline.py "$f"
            gzip -f "$f"; cat gpurun_out/trace_$tag/timeline.txt ;;
        skinny) step 300 gpurun_out/skinny.jsonl python -u scripts/bench_skinny.py ;;
        skinnyhot) step 300 gpurun_out/skinny_hot.jsonl python -u scripts/bench_skinny.py --batches 1 --cold-mb 1 --T 150
                   step 300 gpurun_out/skinny_cold.jsonl python -u scripts/bench_skinny.py --batches 1 --cold-mb 512 --T 150 ;;
        attn) step 300 gpurun_out/attn.jsonl python -u scripts/bench_skinny.py --attn-only --batches 1,8,32 --T 150,1024 ;;
        pgemm) step 300 gpurun_out/pgemm.jsonl python -u scripts/bench_prefill_gemm.py; grep '^{' gpurun_out/pgemm.jsonl ;;
        pgemmt:*)  # pgemmt:<tile ids, ','>  the same plus forced tile configs (max rel err vs fp32 each)
            step 400 gpurun_out/pgemm.jsonl python -u scripts/bench_prefill_gemm.py --tiles "${task#pgemmt:}"
            grep '^{' gpurun_out/pgemm.jsonl ;;
        conc) step 300 gpurun_out/conc.jsonl python -u scripts/bench_concurrency.py; grep '^{' gpurun_out/conc.jsonl ;;
        ps) step 300 gpurun_out/ps.jsonl python -u scripts/bench_ps.py --ops lmhead --batches 256,512,1024 ;;
        pst:*)  # pst:<tile ids, ','>  LM head at 512 rows: gemm_ps vs forced tiled configs
            step 300 gpurun_out/ps.jsonl python -u scripts/bench_ps.py --ops lmhead --batches 512 --tiles "${task#pst:}"
            grep '^{' gpurun_out/ps.jsonl ;;
        gate) step 300 gpurun_out/gate.jsonl python -u scripts/bench_gate.py --clients 100 --rounds 5 ;;
        serving5) step 300 gpurun_out/serving5.jsonl python -u scripts/bench_serving.py --rates 5 --queries 100 \
                      --modes continuous --prompt-jitter 0; grep '^{' gpurun_out/serving5.jsonl ;;
        serving) step 400 gpurun_out/serving.jsonl python -u scripts/bench_serving.py --rates 20,200,1000 --queries 400 \
                     --modes continuous; grep '^{' gpurun_out/serving.jsonl ;;
        tpprof:*)  # tpprof:<tag>:<model>:<tp>  TP ranks sharing cuda:0 under rocprofv3 (one kernel_stats per rank)
            spec=${task#tpprof:}; tag=${spec%%:*}; rest=${spec#*:}; model=${rest%%:*}; tpn=${rest#*:}
            export TMPDIR=/tmp; D=gpurun_out/tpprof_$tag; mkdir -p $D
            step 600 $D/run.log rocprofv3 --kernel-trace --stats -d $D -o run_%pid% --output-format csv \
                -- python3 scripts/tp_shared_gpu.py --model "$model" --tp "$tpn" --batch 1 --reps 2
            find $D -name "*_kernel_trace.csv" -delete
            for f in $(find $D -name "*kernel_stats.csv"); do python scripts/kstats.py "$f" > "${f%.csv}.summary.txt"; done
            grep '^{' $D/run.log; head -14 $(find $D -name "*kernel_stats.summary.txt" | head -1) ;;
        dftrace:*)  # dftrace:<tag>:<batch>[:ENV=v,...]  in-kernel phase trace of the dataflow decode -> gpurun_out/dftrace_<tag>.json
            spec=${task#dftrace:}; tag=${spec%%:*}; rest=${spec#*:}; b=${rest%%:*}; envs=""
            [[ $rest == *:* ]] && envs=${rest#*:}
            step 300 gpurun_out/dftrace_$tag.log env ${envs//,/ } python -u scripts/df_trace.py --model gpt2 --batch "$b" \
                --out gpurun_out/dftrace_$tag.json
            tail -2 gpurun_out/dftrace_$tag.log | cut -c1-300 ;;
        dfsweep:*)  # dfsweep:<df_sweep.sh args, ';' for spaces>  e.g. dfsweep:-b;1,2;default;DLMS_DF_J=1
            spec=${task#dfsweep:}
            step 900 gpurun_out/dfsweep.log bash scripts/df_sweep.sh -o gpurun_out/df_sweep.jsonl ${spec//;/ }
            tail -12 gpurun_out/dfsweep.log ;;
        grpc:*)  # grpc:<tutoring|lms>:<rates>[:<ENV=v,...>]  sustained open-loop gRPC serving -> gpurun_out/grpc.jsonl
            spec=${task#grpc:}; tgt=${spec%%:*}; rest=${spec#*:}; rates=${rest%%:*}; envs=""
            if [ "$rest" != "$rates" ]; then envs=${rest#*:}; fi
            step 600 gpurun_out/grpc.log env ${envs//,/ } python -u scripts/bench_grpc.py --target "$tgt" --rates "$rates" \
                --duration 20 --warmup 8 --client-procs 8 --out gpurun_out/grpc.jsonl --log gpurun_out/grpc_server.log \
                --tag "$envs"
            tail -2 gpurun_out/grpc.jsonl | cut -c1-400 ;;
        e2e:*) step 900 gpurun_out/e2e_${task#e2e:}.log python -u scripts/run_config.py --config ${task#e2e:}
               tail -3 gpurun_out/e2e_${task#e2e:}.log ;;
        e2e1:*) step 900 gpurun_out/e2e_${task#e2e1:}_tp1.log python -u scripts/run_config.py --config ${task#e2e1:} --tp 1
                tail -3 gpurun_out/e2e_${task#e2e1:}_tp1.log ;;
        sweep:*)
            IFS=';' read -ra sets <<< "${task#sweep:}"
            for envs in "${sets[@]}"; do
                ev=${envs//,/ }; if [ "$ev" = "default" ]; then ev=""; fi
                step 300 gpurun_out/sweep.log env $ev python -u bench.py --steps 5 --warmup 2 --latency-batches ""
                echo "{\"env\": \"$envs\", \"bench\": $(grep '^{' gpurun_out/sweep.log | tail -1)}" >> gpurun_out/sweep.jsonl
                tail -1 gpurun_out/sweep.jsonl
            done ;;
        sweep1:*|sweep4:*|sweep32:*)  # the same at batch 1 and 2 / 3 and 4 / 16 and 32: p50 per query
            IFS=';' read -ra sets <<< "${task#*:}"
            bs="1 2"; [[ $task == sweep32:* ]] && bs="16 32"; [[ $task == sweep4:* ]] && bs="3 4"
            for envs in "${sets[@]}"; do
                for b in $bs; do
                    step 300 gpurun_out/sweep1.log env ${envs//,/ } python -u bench.py --batch $b --steps 8 --warmup 2 --latency-batches ""
                    echo "{\"env\": \"$envs\", \"batch\": $b, \"bench\": $(grep '^{' gpurun_out/sweep1.log | tail -1)}" >> gpurun_out/sweep1.jsonl
                done
            done
            python -c "import json; [print(d['env'], d['batch'], d['bench']['p50_query_latency_ms']) for d in map(json.loads, open('gpurun_out/sweep1.jsonl'))]" ;;
        *) echo "unknown task $task" >&2; exit 2 ;;
    esac
done
