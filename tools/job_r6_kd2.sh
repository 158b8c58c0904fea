#!/bin/bash
# Round 6: k1d configs whose ring holds a unit's whole input (D = K / KC + 1), their tests, and timings on
# the big-pixel 1x1 ops; with the instrumented library the same configs with the epilogue's stores
# dropped (xkd*_nostore: does a ring wait queue behind the previous unit's stores?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_k1s.py -k "kd" \
  > gpurun_out/kd2_tests.log 2>&1 || { tail -30 gpurun_out/kd2_tests.log; exit 1; }
tail -2 gpurun_out/kd2_tests.log
args=""
for s in 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 20,192,28,28,96 1,96,256,256,96; do
  args="$args --conv $s,1,1,1,1,0,0"
done
timeout -k 10 600 python -u tools/cfgprobe.py $args --cfg kd --splits 0,8 --json gpurun_out/kd2_probe.json \
  > gpurun_out/kd2_probe.log 2>&1 || { tail -30 gpurun_out/kd2_probe.log; exit 1; }
timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 \
  --conv 5,96,54,54,96,1,1,1,1,0,0 --cfg xkd --splits 0 > gpurun_out/kd2_diag.log 2>&1
rc=$?; grep -v unsupported gpurun_out/kd2_probe.log | awk '/tuned/ || /S=\+0/'; cat gpurun_out/kd2_diag.log; exit $rc
