#!/bin/bash
# wgx stage skeleton: pure-MFMA diagnostic builds (instrumented library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S43="20 64 56 56 192 3 3 1 1 1 1"
A=()
for c in xwx43_onlymfma xwx43_puremfma xwx43_puremfma_nobar xwx43_nodmaissue xwx43_nodma wx43s12; do
  A+=(kt_$c 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "$S43" --cfg $c ::)
done
tools/gpu_job.sh "${A[@]}" true 5 true
