set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ab
mkdir -p $L
for b in 1024 256 512 2048; do
  timeout -k 10 300 python bench.py --batch $b --steps 4 --warmup 1 > $L/bench_b$b.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_b$b.log; exit 1; }
  echo "batch=$b $(tail -1 $L/bench_b$b.log | cut -c90-190)"
done
timeout -k 10 300 python bench.py --weight-dtype fp8 --steps 4 --warmup 1 > $L/bench_fp8.log 2>&1 || { echo "fp8 rc=$?"; exit 1; }
echo "fp8 $(tail -1 $L/bench_fp8.log | cut -c90-190)"
scripts/prof_bench.sh ab1024 --steps 3 --warmup 1 || exit 1
echo ALLDONE
