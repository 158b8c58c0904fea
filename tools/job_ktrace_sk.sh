#!/bin/bash
# Round 5: in-kernel timelines (instrumented library) of the stream-K wx routes (last-arriver tails?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ktrace.py --reps 3 \
  --conv "20 384 13 13 256 3 3 1 1 1 1" --conv "5 96 27 27 256 5 5 1 1 2 2" --conv "1 256 122 122 384 3 3 1 1 1 1" \
  --conv "1 256 57 57 384 3 3 1 1 1 1" --conv "20 144 14 14 288 3 3 1 1 1 1" --conv "20 160 14 14 320 3 3 1 1 1 1" \
  > gpurun_out/ktrace_sk.log 2>&1
