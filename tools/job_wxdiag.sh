#!/bin/bash
# wgx stage decomposition: diagnostic builds (instrumented library) beside the real configs, per-block
# device-clock marks (tools/ktrace.py: m1-2 = the stage loop, m2-4 = the epilogue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S43="20 64 56 56 192 3 3 1 1 1 1"
S25="20 96 27 27 256 5 5 1 1 2 2"
A=()
for c in wx43s12 xwx43_noxf xwx43_nomfma xwx43_nodma xwx43_nou xwx43_novf xwx43_nobar xwx43_onlymfma xwx43_onlyxf; do
  A+=(kt_$c 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "$S43" --cfg $c ::)
done
for c in wx25s6 xwx25_noxf xwx25_nomfma xwx25_nou xwx25_onlymfma; do
  A+=(kt_$c 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "$S25" --cfg $c ::)
done
tools/gpu_job.sh "${A[@]}" wgxtest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgx.py
