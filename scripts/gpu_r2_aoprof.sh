#!/bin/bash
cd "$GRAFT_REPO_ROOT"
DLMS_FUSE_ATTN_OPROJ=1 bash scripts/prof_bench.sh b1_ao --batch 1 --steps 2 --warmup 1 --latency-batches ""
