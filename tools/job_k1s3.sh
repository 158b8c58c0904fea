#!/bin/bash
# k1s staged epilogue: parity, alignment fallbacks, decomposition, probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OPS=()
for d in 20,96,54,54,96 20,64,56,56,64 20,256,27,27,256 20,256,28,28,128 20,192,28,28,96 20,256,28,28,64 \
         20,192,28,28,64 20,192,28,28,32 20,384,13,13,384 5,96,54,54,96 5,64,56,56,64 5,256,27,27,256; do
  OPS+=(--conv "$d,1,1,1,1,0,0")
done
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_k1s.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "ks_ or dword" :: \
  diag 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 --cfg xks --splits 1,2 :: \
  probe 500 python -u tools/cfgprobe.py "${OPS[@]}" --cfg ks --splits 1,2 --json gpurun_out/k1s_probe.json
