set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1u
mkdir -p $L
scripts/gpu_step.sh 600 $L/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
scripts/gpu_step.sh 200 $L/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py || exit 1
scripts/prof_bench.sh u1024 --steps 3 --warmup 1 || exit 1
echo ALLDONE
