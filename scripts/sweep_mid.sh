cd $GRAFT_REPO_ROOT
for envs in "X=1" "DLMS_SMALL_MAX_ROWS=1" "DLMS_MID_STREAMS=2"; do
  timeout -k 10 300 env $envs python -u bench.py --batch 64 --steps 3 --warmup 1 --latency-batches 2,4,8,16,32,48 > gpurun_out/sw.log 2>&1 || exit 1
  echo "{\"env\": \"$envs\", \"bench\": $(grep '^{' gpurun_out/sw.log | tail -1)}" >> gpurun_out/sweep_mid.jsonl
done
