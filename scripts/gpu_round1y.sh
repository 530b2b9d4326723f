set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1y
mkdir -p $L
for sm in 1 2 3 2 1; do
  DLMS_SPLIT_MAX=$sm timeout -k 10 200 python bench.py --steps 4 --warmup 1 > $L/bench_split$sm.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_split$sm.log; exit 1; }
  echo "split_max=$sm $(tail -1 $L/bench_split$sm.log | cut -c1-160)"
done
echo ALLDONE
