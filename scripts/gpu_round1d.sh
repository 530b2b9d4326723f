set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1d
mkdir -p $L
scripts/gpu_step.sh 400 $L/tests.log python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -p no:cacheprovider || exit 1
scripts/gpu_step.sh 300 $L/kbench.log python scripts/bench_kernels.py || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py --steps 3 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench_b512.log python bench.py --steps 3 --warmup 1 --batch 512 || exit 1
echo ALLDONE
