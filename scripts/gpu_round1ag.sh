set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ag
mkdir -p $L
timeout -k 10 400 python scripts/bench_kernels.py --batches=32768 --tiles=-1,3,6,8,9,10,11,12,13 --vendor --ops qkv,fc,proj > $L/prefill_tiles.log 2>&1 || { echo "rc=$?"; tail -20 $L/prefill_tiles.log; exit 1; }
grep '^{' $L/prefill_tiles.log | cut -c1-140
echo ALLDONE
