set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1p
mkdir -p $L
scripts/gpu_step.sh 600 $L/kbench.log python scripts/bench_kernels.py --batches=256,1024,2048 --tiles=-1,6,12,13,8,10,2 --ops fc,lmhead || exit 1
echo ALLDONE
