#!/bin/bash
# Winograd parity, then every wg* config on conv-set shapes in one process (same-box comparison)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in ${WG_OPS:-20,64,56,56,192 20,384,13,13,384 20,144,14,14,288 20,384,6,6,1024 20,128,28,28,192 20,256,56,56,256}; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  probe 400 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits ${SPLITS:-11,15} --json gpurun_out/wg_probe.json
