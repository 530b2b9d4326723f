set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1s
mkdir -p $L
scripts/gpu_step.sh 400 $L/kbench.log python scripts/bench_kernels.py --batches=1024,256 --tiles=-1 --ops attn || exit 1
scripts/gpu_step.sh 900 $L/tests.log python -m pytest tests -m gpu -q -x -p no:cacheprovider || exit 1
echo ALLDONE
