#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in "20 3 227 227 96 11 11 4 4 0 0" "20 3 224 224 64 7 7 2 2 3 3" "5 3 227 227 96 11 11 4 4 0 0" "20 832 7 7 256 1 1 1 1 0 0" "5 832 7 7 48 1 1 1 1 0 0" "1 160 7 7 320 3 3 1 1 1 1"; do
  timeout -k 10 60 python tools/ktrace.py --conv "$s" --reps 3 >> gpurun_out/kt2.log 2>&1 || exit $?
done
