#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "20 384 13 13 384 3 3 1 1 1 1" "20 64 56 56 192 3 3 1 1 1 1" "20 96 27 27 256 5 5 1 1 2 2" "20 3 227 227 96 11 11 4 4 0 0"; do
  timeout -k 10 60 python tools/ktrace.py --conv "$s" --reps 3 >> gpurun_out/kt3.log 2>&1 || exit $?
done
