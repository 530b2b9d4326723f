set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1t
mkdir -p $L
for v in 0 2 0 2; do
DLMS_ATTN_VARIANT=$v scripts/gpu_step.sh 300 $L/bench_v$v.log python bench.py --steps 4 --warmup 1 || exit 1
done
DLMS_ATTN_VARIANT=2 scripts/gpu_step.sh 300 $L/bench_b256_v2.log python bench.py --batch 256 --steps 5 --warmup 1 || exit 1
scripts/gpu_step.sh 300 $L/bench_b256_v0.log python bench.py --batch 256 --steps 5 --warmup 1 || exit 1
echo ALLDONE
