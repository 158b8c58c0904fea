#!/bin/bash
# Winograd parity, wgp vs wgi (interleaved stage) times on conv-set shapes, per-phase clocks (trace build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in 20,64,56,56,192 20,384,13,13,384 20,256,13,13,384 20,144,14,14,288 20,384,6,6,1024 20,96,28,28,128 20,256,56,56,256; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  probe 300 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits 1,11,15 --json gpurun_out/wg_probe.json :: \
  ph1 120 env BH_LIB_NAME=libboda_hip_wgkt.so python -u tools/wg_phases.py --conv 20,64,56,56,192,3,3,1,1,1,1 --cfg wgp64x64v --cfg wgi64x64v --splits 15 :: \
  ph2 120 env BH_LIB_NAME=libboda_hip_wgkt.so python -u tools/wg_phases.py --conv 20,384,13,13,384,3,3,1,1,1,1 --cfg wgp128x32 --cfg wgi128x32 --splits 11
