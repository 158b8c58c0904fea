#!/bin/bash
# Winograd configs (wg*): parity tests, then their times on the conv set's 3x3 stride-1 ops
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in 20,64,56,56,192 20,384,13,13,384 20,256,13,13,384 20,128,28,28,192 20,384,13,13,256 20,144,14,14,288 \
         20,160,14,14,320 20,384,6,6,1024 20,96,28,28,128 20,192,7,7,384 5,384,13,13,384 5,128,28,28,192 5,64,56,56,192; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  probe 500 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits ${SPLITS:-0,2,5} --json gpurun_out/wg_probe.json
