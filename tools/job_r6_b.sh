#!/bin/bash
# Round 6: (1) the resident-bank 1x1 kernels with the epilogue's stores dropped (instrumented library,
# xkn* / xks* configs) next to their table routes: how much of a unit's time is a ring wait queued behind
# the previous unit's stores; (2) retune of the 3x3 stride-1 ops against the lean-transform Winograd
# configs, then a same-box table A B A B (tools/job_r6_retune.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 \
  --conv 1,96,256,256,96,1,1,1,1,0,0 --conv 20,64,57,57,64,1,1,1,1,0,0 --cfg xkn --cfg xks --splits 1,8 \
  > gpurun_out/kn_nostore.log 2>&1 || { tail -20 gpurun_out/kn_nostore.log; exit 1; }
timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 \
  --conv 1,96,256,256,96,1,1,1,1,0,0 --conv 20,64,57,57,64,1,1,1,1,0,0 --cfg kn32p32c32q3w8 --cfg kn32p32c16q4w8 \
  --cfg kn96p64c8q4w4 --cfg ks96c32q3 --splits 1,8 > gpurun_out/kn_store.log 2>&1 || { tail -20 gpurun_out/kn_store.log; exit 1; }
grep -v unsupported gpurun_out/kn_nostore.log; grep -v unsupported gpurun_out/kn_store.log
KEY_RE=' 3 3 1 1 [01] [01]$' CFG_RE='^wgl' MIN_GAIN=0.01 TUNE_SECS=900 bash tools/job_r6_retune.sh
