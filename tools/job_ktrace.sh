#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "5 832 7 7 48 1 1 1 1 0 0" "1 832 7 7 160 1 1 1 1 0 0" "20 832 7 7 256 1 1 1 1 0 0" "1 160 7 7 320 3 3 1 1 1 1" "5 192 7 7 384 3 3 1 1 1 1" "20 512 14 14 112 1 1 1 1 0 0" "1 480 14 14 96 1 1 1 1 0 0"; do
  timeout -k 10 60 python tools/ktrace.py --conv "$s" --reps 3 >> gpurun_out/kt4.log 2>&1 || exit $?
done
timeout -k 10 60 tools/lat_bench >> gpurun_out/kt4.log 2>&1
