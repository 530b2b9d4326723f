set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1r
mkdir -p $L
scripts/gpu_step.sh 300 $L/prof.log rocprofv3 --kernel-trace --stats -d $L/prof1024 -o run -- python3 bench.py --batch 1024 --steps 2 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench.log python bench.py || exit 1
echo ALLDONE
