set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1z
mkdir -p $L
for b in 256 64; do
for sm in 8 2 3 8 2; do
  DLMS_SPLIT_MAX=$sm timeout -k 10 200 python bench.py --batch $b --steps 4 --warmup 1 > $L/bench_b${b}_split$sm.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_b${b}_split$sm.log; exit 1; }
  echo "batch=$b split_max=$sm $(tail -1 $L/bench_b${b}_split$sm.log | cut -c90-200)"
done
done
echo ALLDONE
