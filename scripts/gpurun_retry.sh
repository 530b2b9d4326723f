#!/bin/bash
# gpurun_retry.sh <out file> <timeout s> <command>: one gpurun call, re-submitted (after 150 s) only while
# the pool reports "transient" (no box / busy slots / box died while being prepared: nothing ran, nothing
# charged).  A call whose command ran -- pass or fail -- is never repeated.
out=$1; tmo=$2; cmd=$3
for i in $(seq 1 ${GPURUN_TRIES:-8}); do
    /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$out" 2>&1
    st=$(python3 -c "import json; print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status', ''))" 2>/dev/null)
    [ "$st" = "transient" ] || exit 0
    echo "[retry $i: transient]" >> "$out.retries"
    sleep 150
done
