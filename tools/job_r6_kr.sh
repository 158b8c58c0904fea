#!/bin/bash
# Round 6: the register-bank 1x1 kernel (k1r, kr* configs): tests, then timings next to the table routes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_k1s.py -k "kr" \
  > gpurun_out/kr_tests.log 2>&1 || { tail -40 gpurun_out/kr_tests.log; exit 1; }
tail -2 gpurun_out/kr_tests.log
args=""
for s in 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 20,192,28,28,96 20,192,28,28,64 20,192,28,28,32 \
         20,192,28,28,16 5,192,28,28,96 5,192,28,28,64 1,192,28,28,64 1,96,54,54,96 1,64,56,56,64 20,64,57,57,64 \
         1,96,256,256,96 20,128,28,28,128; do
  args="$args --conv $s,1,1,1,1,0,0"
done
timeout -k 10 600 python -u tools/cfgprobe.py $args --cfg kr --splits 1,2,8 --json gpurun_out/kr_probe.json \
  > gpurun_out/kr_probe.log 2>&1 || { tail -30 gpurun_out/kr_probe.log; exit 1; }
grep -v unsupported gpurun_out/kr_probe.log
