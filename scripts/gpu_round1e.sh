set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1e
mkdir -p $L
scripts/gpu_step.sh 500 $L/tests.log python -m pytest tests -m gpu -q -p no:cacheprovider || exit 1
scripts/gpu_step.sh 300 $L/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py --steps 3 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench_b512.log python bench.py --steps 3 --warmup 1 --batch 512 || exit 1
scripts/gpu_step.sh 300 $L/prof.log rocprofv3 --kernel-trace --stats -d $L/prof -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --batch 256 || exit 1
echo ALLDONE
