set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1af
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $L/engine_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $L/engine_tests.log; exit 1; }
tail -1 $L/engine_tests.log
timeout -k 10 400 python -u scripts/bench_serving.py --rates 2000,4000,6000 --queries 6000 --max-batch 1024 --modes continuous > $L/serving_1024.log 2>&1 || { echo "rc=$?"; tail -20 $L/serving_1024.log; exit 1; }
grep '^{' $L/serving_1024.log | cut -c1-200
timeout -k 10 400 python -u scripts/bench_serving.py --rates 6000 --queries 6000 --max-batch 1024 --modes continuous --chunk 4 > $L/serving_1024_c4.log 2>&1 || { echo "rc=$?"; tail -20 $L/serving_1024_c4.log; exit 1; }
grep '^{' $L/serving_1024_c4.log | cut -c1-200
echo ALLDONE
