#!/bin/bash
# Round 6: 1x1 configs with a unit's whole K in flight (kn*q12 / kn*q6, kw*q12 / kw*q6): tests, then
# timings next to the table routes on the K = 96 big-pixel ops
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_k1s.py \
  -k "q12 or q6" > gpurun_out/deep_tests.log 2>&1 || { tail -30 gpurun_out/deep_tests.log; exit 1; }
tail -2 gpurun_out/deep_tests.log
args=""
for s in 20,96,54,54,96 5,96,54,54,96 20,192,28,28,96 1,96,256,256,96 20,96,55,55,96; do
  args="$args --conv $s,1,1,1,1,0,0"
done
timeout -k 10 600 python -u tools/cfgprobe.py $args --cfg kn32p32c8q12 --cfg kn32p32c16q6 --cfg kw96c8q12 --cfg kw96c16q6 \
  --cfg kw32c8q12 --splits 1,2,8 --json gpurun_out/deep_probe.json > gpurun_out/deep_probe.log 2>&1 \
  || { tail -30 gpurun_out/deep_probe.log; exit 1; }
grep -v unsupported gpurun_out/deep_probe.log
