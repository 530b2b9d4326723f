set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1k
mkdir -p $L
for b in 256 256 512; do
scripts/gpu_step.sh 300 $L/bench.log python bench.py --batch $b --steps 10 --warmup 2 || exit 1
done
scripts/gpu_step.sh 300 $L/prof.log rocprofv3 --kernel-trace --stats -d $L/prof256 -o run -- python3 bench.py --batch 256 --steps 3 --warmup 1 || exit 1
echo ALLDONE
