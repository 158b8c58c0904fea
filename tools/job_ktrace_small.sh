#!/bin/bash
# In-kernel timelines (instrumented library, tools/ktrace.py) of small / mid conv ops on their table
# routes: where a 3-25 us op's time goes (entry, first operands, K loop, split-K ticket, drained stores)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ktrace.py --reps 4 \
  --conv "1 384 13 13 384 3 3 1 1 1 1" --conv "5 384 13 13 384 3 3 1 1 1 1" --conv "20 192 7 7 384 3 3 1 1 1 1" \
  --conv "20 528 14 14 128 1 1 1 1 0 0" --conv "1 832 7 7 32 1 1 1 1 0 0" --conv "5 528 14 14 160 1 1 1 1 0 0" \
  --conv "1 96 27 27 256 5 5 1 1 2 2" --conv "5 192 28 28 96 1 1 1 1 0 0" --conv "20 528 14 14 160 1 1 1 1 0 0" \
  --conv "1 64 56 56 192 3 3 1 1 1 1" --conv "20 1024 6 6 1000 1 1 1 1 0 0" > gpurun_out/ktrace_small.log 2>&1
