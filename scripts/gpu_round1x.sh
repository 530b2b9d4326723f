set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1x
mkdir -p $L
timeout -k 10 200 python -u -m pytest tests/test_kernel_checks_gpu.py -x -v -s --timeout 150 --timeout-method thread > $L/checks.log 2>&1 || { echo "checks rc=$?"; tail -40 $L/checks.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $L/pytest_gpu.log 2>&1 || { echo "gpu rc=$?"; tail -40 $L/pytest_gpu.log; exit 1; }
tail -3 $L/pytest_gpu.log
timeout -k 10 300 python bench.py > $L/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench.log; exit 1; }
tail -1 $L/bench.log
echo ALLDONE
