set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1w
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v -s --timeout 240 --timeout-method thread > $L/xgmi.log 2>&1 || { echo "xgmi rc=$?"; tail -30 $L/xgmi.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py -x -v -s --timeout 300 --timeout-method thread > $L/tp.log 2>&1 || { echo "tp rc=$?"; tail -30 $L/tp.log; exit 1; }
tail -5 $L/xgmi.log; tail -5 $L/tp.log
echo ALLDONE
