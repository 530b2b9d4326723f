set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1l
mkdir -p $L
scripts/gpu_step.sh 900 $L/kbench.log python scripts/bench_kernels.py --batches=256,64,1024 --tiles=-1,0,1,4,7,2,5,3 --ops qkv,oproj,fc,proj,lmhead || exit 1
echo ALLDONE
