set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1m
mkdir -p $L
scripts/gpu_step.sh 400 $L/tests.log python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x -p no:cacheprovider || exit 1
for b in 256 64 1024; do
scripts/gpu_step.sh 300 $L/bench.log python bench.py --batch $b --steps 10 --warmup 2 || exit 1
done
scripts/gpu_step.sh 300 $L/prof.log rocprofv3 --kernel-trace --stats -d $L/prof256 -o run -- python3 bench.py --batch 256 --steps 3 --warmup 1 || exit 1
scripts/gpu_step.sh 600 $L/cfg2.log python scripts/run_config.py --config 2 --students 64 --queries 2 --workdir /tmp/cfg2 || exit 1
echo ALLDONE
