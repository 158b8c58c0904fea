#!/bin/bash
# wgx: parity, phase marks of the two 6x6 forms, wx* times on the conv set's 3x3 / 5x5 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=()
for s in 20,64,56,56,192,3,3,1,1,1,1 20,128,28,28,192,3,3,1,1,1,1 20,96,28,28,128,3,3,1,1,1,1 \
         20,384,13,13,384,3,3,1,1,1,1 20,96,27,27,256,5,5,1,1,2,2 5,96,27,27,256,5,5,1,1,2,2 \
         20,32,28,28,96,5,5,1,1,2,2 5,64,56,56,192,3,3,1,1,1,1; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  wgxtest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgx.py :: \
  kt43 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 64 56 56 192 3 3 1 1 1 1" --cfg wx43s12 :: \
  kt43o 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 64 56 56 192 3 3 1 1 1 1" --cfg xwx43_onlymfma :: \
  kt25 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 96 27 27 256 5 5 1 1 2 2" --cfg wx25s6 :: \
  wgxprobe 400 python -u tools/cfgprobe.py "${P[@]}" --cfg wx --splits 0 --json gpurun_out/wgxprobe.json
