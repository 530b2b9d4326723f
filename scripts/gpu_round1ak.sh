set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ak
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "argmax or 256" > $L/pytest_argmax.log 2>&1 || { echo "argmax rc=$?"; tail -40 $L/pytest_argmax.log; exit 1; }
tail -2 $L/pytest_argmax.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $L/pytest_gpu.log 2>&1 || { echo "gpu rc=$?"; tail -40 $L/pytest_gpu.log; exit 1; }
tail -2 $L/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $L/bench$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench$i.log; exit 1; }
echo "bench $(tail -1 $L/bench$i.log | cut -c90-190)"
done
echo ALLDONE
