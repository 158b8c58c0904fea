#!/bin/bash
# wgx parity after the residual fix; wgx phase marks (instrumented library); k1s / srk / ring-128
# candidates on the batch-20 1x1 ops
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K1=()
for s in 20,384,13,13,384,1,1,1,1,0,0 20,512,14,14,144,1,1,1,1,0,0 20,96,54,54,96,1,1,1,1,0,0 \
         20,256,27,27,256,1,1,1,1,0,0 20,1024,6,6,1000,1,1,1,1,0,0 20,64,56,56,64,1,1,1,1,0,0 \
         20,256,28,28,128,1,1,1,1,0,0 20,528,14,14,256,1,1,1,1,0,0; do K1+=(--conv "$s"); done
tools/gpu_job.sh \
  wgxtest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgx.py :: \
  kt43 120 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 64 56 56 192 3 3 1 1 1 1" --cfg wx43s12 :: \
  kt25 120 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 96 27 27 256 5 5 1 1 2 2" --cfg wx25s6 :: \
  kt23 120 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 384 13 13 384 3 3 1 1 1 1" --cfg wx23s6w4 :: \
  ks 300 python -u tools/cfgprobe.py "${K1[@]}" --cfg ks --splits 1,2 --json gpurun_out/probe_ks.json :: \
  srk 400 python -u tools/cfgprobe.py "${K1[@]}" --cfg srk --splits 1,2,5,6 --json gpurun_out/probe_srk.json :: \
  r128 300 python -u tools/cfgprobe.py "${K1[@]}" --cfg r128 --splits 1,2,3 --json gpurun_out/probe_r128.json
