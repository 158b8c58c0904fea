#!/bin/bash
# Position-split Winograd (bh_wgx.hip): parity of every wx* config, then wx* times beside the table
# route on the conv set's 3x3 / 5x5 shapes (graph-amortized, tools/cfgprobe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=()
for s in 20,64,56,56,192,3,3,1,1,1,1 20,128,28,28,192,3,3,1,1,1,1 20,96,28,28,128,3,3,1,1,1,1 \
         20,384,13,13,384,3,3,1,1,1,1 20,256,13,13,384,3,3,1,1,1,1 20,160,14,14,320,3,3,1,1,1,1 \
         20,96,27,27,256,5,5,1,1,2,2 5,96,27,27,256,5,5,1,1,2,2 20,32,28,28,96,5,5,1,1,2,2 \
         20,32,14,14,128,5,5,1,1,2,2 5,64,56,56,192,3,3,1,1,1,1; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  wgxtest 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wgx.py :: \
  wgxprobe 400 python -u tools/cfgprobe.py "${P[@]}" --cfg wx --splits 0 --json gpurun_out/wgxprobe.json
