#!/bin/bash
# wgx: parity, then wx* times on chosen 3x3 / 5x5 ops beside the table's route
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=()
for s in ${WX_OPS:-20,64,56,56,192,3,3,1,1,1,1 20,64,57,57,192,3,3,1,1,1,1 1,256,122,122,384,3,3,1,1,0,0 \
         20,128,28,28,192,3,3,1,1,1,1 20,96,28,28,128,3,3,1,1,1,1 20,384,13,13,384,3,3,1,1,1,1 \
         20,384,6,6,1024,3,3,1,1,1,1 5,96,27,27,256,5,5,1,1,2,2 20,96,27,27,256,5,5,1,1,2,2 \
         20,32,28,28,96,5,5,1,1,2,2 5,64,56,56,192,3,3,1,1,1,1}; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  wgxtest 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgx.py :: \
  wxkprobe 600 python -u tools/cfgprobe.py "${P[@]}" --cfg wx --splits 0 --json gpurun_out/wxkprobe.json
