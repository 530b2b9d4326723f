set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ai
mkdir -p $L
timeout -k 10 300 python scripts/bench_kernels.py --batches=512,1024 --vocab 50432 --tiles=-1,6,9,14 --ops lmhead > $L/lmhead256.log 2>&1 || { echo "rc=$?"; tail -20 $L/lmhead256.log; exit 1; }
grep '^{' $L/lmhead256.log | cut -c1-125
timeout -k 10 300 python scripts/bench_kernels.py --batches=2048,4096,8192,16384 --tiles=-1,14 --ops qkv,fc > $L/mid.log 2>&1 || { echo "rc=$?"; tail -20 $L/mid.log; exit 1; }
grep '^{' $L/mid.log | cut -c1-125
echo ALLDONE
