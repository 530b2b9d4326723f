set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1h
mkdir -p $L
scripts/gpu_step.sh 400 $L/kbench.log python scripts/bench_kernels.py --batches=256,1024 --tiles=-1,1,3,4,5 || exit 1
scripts/gpu_step.sh 300 $L/prof.log rocprofv3 --kernel-trace --stats -d $L/prof -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --batch 1024 || exit 1
echo ALLDONE
