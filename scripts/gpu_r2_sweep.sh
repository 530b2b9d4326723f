#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_skinny_gpu.py -k "persist" > gpurun_out/r2_sw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2_sw_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep_bench.sh persist "DLMS_PERSIST_ATTN_BLOCKS=0" "DLMS_PERSIST_ATTN_BLOCKS=256" "DLMS_PERSIST_ATTN_BLOCKS=512" "DLMS_PERSIST_ATTN_BLOCKS=1024" "DLMS_PERSIST_ATTN_BLOCKS=512 DLMS_OVERLAP_PARTS=3" "DLMS_PERSIST_ATTN_BLOCKS=512 DLMS_OVERLAP_SPLIT_CAP=4"
