set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ae
mkdir -p $L
timeout -k 10 400 python -u scripts/bench_serving.py --rates 2000,4000,6000 --queries 6000 --max-batch 1024 --modes continuous > $L/serving_1024.log 2>&1 || { echo "rc=$?"; tail -20 $L/serving_1024.log; exit 1; }
grep '^{' $L/serving_1024.log | cut -c1-200
echo ALLDONE
