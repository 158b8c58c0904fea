#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BH_LIB_NAME=libboda_hip_wgkt.so
tools/gpu_job.sh \
  ph1 120 python -u tools/wg_phases.py --conv 5,384,13,13,384,3,3,1,1,1,1 --cfg wgp128x32 --cfg wgp64x64 --splits 1,5,11 :: \
  ph2 120 python -u tools/wg_phases.py --conv 5,128,28,28,192,3,3,1,1,1,1 --cfg wgp128x32 --cfg wgp64x64 --splits 1,5 :: \
  pr 200 python -u tools/cfgprobe.py --conv 5,384,13,13,384,3,3,1,1,1,1 --conv 5,128,28,28,192,3,3,1,1,1,1 --cfg wgp --splits 1,5,11
