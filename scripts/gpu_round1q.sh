set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1q
mkdir -p $L
for b in 512 768 1024 1536 2048; do
scripts/gpu_step.sh 300 $L/bench.log python bench.py --batch $b --steps 4 --warmup 1 || exit 1
done
scripts/gpu_step.sh 300 $L/bench.log python bench.py --batch 1024 --steps 4 --warmup 1 --weight-dtype fp8 || exit 1
echo ALLDONE
