set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1n
mkdir -p $L
scripts/gpu_step.sh 400 $L/tests.log python -m pytest tests -m gpu -q -x -p no:cacheprovider || exit 1
rocprofv3 -L > $L/counters.txt 2>&1 || true
scripts/gpu_step.sh 560 $L/cfg2.log python scripts/run_config.py --config 2 --students 48 --queries 2 --workdir $L/cfg2 || exit 1
echo ALLDONE
