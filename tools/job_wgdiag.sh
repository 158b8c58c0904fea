#!/bin/bash
# Winograd diagnostic configs (wrong results by design; -DBH_WG_DIAG build lib/libboda_hip_wgdiag.so):
# stage time with U / strips forced L2-resident, beside the real wgp128x32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in 20,64,56,56,192 20,384,13,13,384 20,128,28,28,192 20,256,56,56,256; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
export BH_LIB_NAME=libboda_hip_wgdiag.so
tools/gpu_job.sh \
  d1 200 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wgp128x32 --splits 11,15 :: \
  d2 200 python -u tools/cfgprobe.py "${OPS[@]}" --cfg xwgp --splits 11,15
