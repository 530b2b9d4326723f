set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1v
mkdir -p $L
scripts/gpu_step.sh 300 $L/config3.log python -u scripts/run_config.py --config 3 --students 64 --queries 2 || exit 1
scripts/gpu_step.sh 300 $L/config4_tp1.log python -u scripts/run_config.py --config 4 --tp 1 --students 64 --queries 2 || exit 1
scripts/gpu_step.sh 300 $L/config5_tp1.log python -u scripts/run_config.py --config 5 --tp 1 --students 32 --queries 2 || exit 1
scripts/gpu_step.sh 300 $L/bench_medium.log python bench.py --model gpt2-medium --steps 3 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench_xl.log python bench.py --model gpt2-xl --steps 2 --warmup 1 --batch 512 || exit 1
echo ALLDONE
