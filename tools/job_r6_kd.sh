#!/bin/bash
# Round 6: the k1d (kd*) 1x1 kernel and the lean-transform Winograd configs (wgl*) -- their tests, then
# graph-amortized timings next to the table routes (tools/cfgprobe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_k1s.py -k "kd" \
  tests/test_gpu_nan.py > gpurun_out/kd_tests.log 2>&1 || { tail -30 gpurun_out/kd_tests.log; exit 1; }
tail -3 gpurun_out/kd_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wino.py -k "wgl" \
  > gpurun_out/wgl_tests.log 2>&1 || { tail -30 gpurun_out/wgl_tests.log; exit 1; }
tail -3 gpurun_out/wgl_tests.log
args=""
for s in 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 20,192,28,28,96 20,256,28,28,128 20,256,28,28,64 \
         20,192,28,28,64 20,192,28,28,32 20,256,28,28,32 20,192,28,28,16 5,256,28,28,64 5,192,28,28,96; do
  args="$args --conv $s,1,1,1,1,0,0"
done
timeout -k 10 600 python -u tools/cfgprobe.py $args --cfg kd --splits 0,1,2,8 --json gpurun_out/kd_probe.json \
  > gpurun_out/kd_probe.log 2>&1 || { tail -30 gpurun_out/kd_probe.log; exit 1; }
args=""
for s in 20,384,13,13,384 20,256,13,13,384 20,128,28,28,192 20,384,6,6,1024 5,64,56,56,192 20,96,28,28,128 \
         20,144,14,14,288 20,160,14,14,320 20,128,14,14,256 20,112,14,14,224 20,384,13,13,256; do
  args="$args --conv $s,3,3,1,1,1,1"
done
timeout -k 10 900 python -u tools/cfgprobe.py $args --cfg wg --splits 1,5,11,21,31 --json gpurun_out/wgl_probe.json \
  > gpurun_out/wgl_probe.log 2>&1
rc=$?; grep -v "unsupported" gpurun_out/kd_probe.log | tail -60; [ $rc -eq 0 ] && timeout -k 10 700 bash tools/opsprof_op37.sh; exit $rc
