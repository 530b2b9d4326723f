set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1al
mkdir -p $L
P=$GRAFT_REPO_ROOT/distributed_lms_raft_llm_amd/ops/_lib/libdlms_hip_noarg.so
n=0
for v in noarg new noarg new noarg new; do
  n=$((n+1))
  if [ $v = noarg ]; then export DLMS_HIP_LIB=$P; else unset DLMS_HIP_LIB; fi
  timeout -k 10 200 python bench.py --steps 6 --warmup 1 > $L/bench_${v}_$n.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_${v}_$n.log; exit 1; }
  echo "bench $v $(tail -1 $L/bench_${v}_$n.log | cut -c20-140)"
done
echo ALLDONE
