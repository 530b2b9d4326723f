set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1aa
mkdir -p $L
for t in none 4 1 7 2 5 none; do
  if [ $t = none ]; then unset DLMS_GEMM_TILE; else export DLMS_GEMM_TILE=$t; fi
  timeout -k 10 200 python bench.py --steps 4 --warmup 1 > $L/bench_tile$t.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_tile$t.log; exit 1; }
  echo "tile=$t $(tail -1 $L/bench_tile$t.log | cut -c90-190)"
done
unset DLMS_GEMM_TILE
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $L/engine_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $L/engine_tests.log; exit 1; }
tail -2 $L/engine_tests.log
echo ALLDONE
