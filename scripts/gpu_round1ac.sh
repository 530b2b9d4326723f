set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ac
mkdir -p $L
for cfg in "512 1024" "512 512" "256 1024" "256 256" "512 512" "512 1024" "2048 1024"; do
  set -- $cfg
  DLMS_OVERLAP_MIN_BATCH=$2 timeout -k 10 300 python bench.py --batch $1 --steps 4 --warmup 1 > $L/bench_b$1_m$2.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  echo "batch=$1 min=$2 $(tail -1 $L/bench_b$1_m$2.log | cut -c90-190)"
done
echo ALLDONE
