#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault/abort/timeout
# (exit >= 124 or a signal), continue on ordinary test failures (exit 1).
# usage: scripts/gpu_step.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
echo "=== $(date +%T) $*" >> "$log"
timeout -k 10 "$secs" "$@" >> "$log" 2>&1
rc=$?
echo "=== rc=$rc" >> "$log"
if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then
  echo "FATAL step rc=$rc: $*" >&2
  exit 99
fi
exit 0
