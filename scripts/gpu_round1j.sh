set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1j
mkdir -p $L
scripts/gpu_step.sh 600 $L/tests.log python -m pytest tests -m gpu -q -x -p no:cacheprovider || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py --batch 1024 --steps 5 --warmup 2 || exit 1
scripts/gpu_step.sh 500 $L/serving.log python scripts/bench_serving.py --rates 200,1000,2000 --queries 3000 || exit 1
echo ALLDONE
