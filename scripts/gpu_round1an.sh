set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1an
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $L/pytest_kernels.log 2>&1 || { echo "kernels rc=$?"; tail -40 $L/pytest_kernels.log; exit 1; }
tail -1 $L/pytest_kernels.log
P=$GRAFT_REPO_ROOT/distributed_lms_raft_llm_amd/ops/_lib/libdlms_hip_old.so
n=0
for cfg in "gpt2-medium 1024" "gpt2-xl 512" "gpt2 1024"; do
  set -- $cfg
  for v in old new old new; do
    n=$((n+1))
    if [ $v = old ]; then export DLMS_HIP_LIB=$P; else unset DLMS_HIP_LIB; fi
    timeout -k 10 200 python bench.py --model $1 --batch $2 --steps 2 --warmup 1 > $L/bench_$1_${v}_$n.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_$1_${v}_$n.log; exit 1; }
    echo "bench $1 $v $(tail -1 $L/bench_$1_${v}_$n.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
echo ALLDONE
