set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ad
mkdir -p $L
timeout -k 10 300 python scripts/bench_kernels.py --batches=512 --tiles=-1,3,5,12 --vendor --ops lmhead > $L/lmhead.log 2>&1 || { echo "rc=$?"; tail -20 $L/lmhead.log; exit 1; }
grep '^{' $L/lmhead.log | cut -c1-150
echo ALLDONE
