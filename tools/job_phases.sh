#!/bin/bash
# Winograd parity, wg* times on conv-set shapes, a PMC pass of one Winograd op
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in 20,64,56,56,192 20,384,13,13,384 20,256,13,13,384 20,144,14,14,288 20,384,6,6,1024 20,96,28,28,128 20,256,56,56,256; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  probe 300 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits ${SPLITS:-1,11,15} --json gpurun_out/wg_probe.json :: \
  pmc 400 tools/pmc.sh gpurun_out/pmcw python3 tools/profile_op.py conv ${PMC_OP:-20,384,13,13,384,3,3,1,1,1,1} --iters 20
