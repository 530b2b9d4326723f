cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/prefill_probe.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_dataflow_gpu.py tests/test_scheduler.py > gpurun_out/t_df.log 2>&1; rc=$?; tail -3 gpurun_out/t_df.log; [ $rc -ne 0 ] && exit $rc
bash scripts/prefill_probe.sh
