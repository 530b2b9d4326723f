set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ah
mkdir -p $L
P=$GRAFT_REPO_ROOT/distributed_lms_raft_llm_amd/ops/_lib/libdlms_hip_prio.so
timeout -k 10 300 python scripts/bench_kernels.py --batches=32768 --tiles=-1,9,14 --ops qkv,fc > $L/prefill_base.log 2>&1 || { echo "rc=$?"; tail -20 $L/prefill_base.log; exit 1; }
DLMS_HIP_LIB=$P timeout -k 10 300 python scripts/bench_kernels.py --batches=32768 --tiles=-1,9,14 --ops qkv,fc > $L/prefill_prio.log 2>&1 || { echo "rc=$?"; tail -20 $L/prefill_prio.log; exit 1; }
echo BASE; grep '^{' $L/prefill_base.log | grep -v split2 | grep -v split4 | grep -v split8 | cut -c1-120
echo PRIO; grep '^{' $L/prefill_prio.log | grep -v split2 | grep -v split4 | grep -v split8 | cut -c1-120
for v in base prio base prio; do
  if [ $v = prio ]; then export DLMS_HIP_LIB=$P; else unset DLMS_HIP_LIB; fi
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 > $L/bench_$v.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "bench $v $(tail -1 $L/bench_$v.log | cut -c90-190)"
done
echo ALLDONE
