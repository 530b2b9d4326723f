set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1i
mkdir -p $L
scripts/gpu_step.sh 500 $L/tests.log python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider || exit 1
scripts/gpu_step.sh 600 $L/kbench.log python scripts/bench_kernels.py --batches=1024,256 --tiles=-1,1,2,3,4,6,8,9,10,11 || exit 1
echo ALLDONE
