set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1g
mkdir -p $L
scripts/gpu_step.sh 600 $L/tests.log python -m pytest tests -m gpu -q -p no:cacheprovider || exit 1
scripts/gpu_step.sh 400 $L/kbench.log python scripts/bench_kernels.py --batches 256,1024 --tiles -1,1,3,4,5 || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py --steps 3 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench_b512.log python bench.py --steps 3 --warmup 1 --batch 512 || exit 1
scripts/gpu_step.sh 300 $L/bench_b1024.log python bench.py --steps 3 --warmup 1 --batch 1024 || exit 1
scripts/gpu_step.sh 300 $L/bench_b2048.log python bench.py --steps 2 --warmup 1 --batch 2048 || exit 1
echo ALLDONE
