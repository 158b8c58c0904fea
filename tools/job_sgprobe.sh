#!/bin/bash
# SGEMM: ring configs on the big sgemm-ops-full shapes beside the table's route
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=()
for m in ${SG_SIZES:-10240 12288 8192}; do S+=(--sgemm "$m,$m,$m"); done
tools/gpu_job.sh \
  sgr 900 python -u tools/cfgprobe.py "${S[@]}" --cfg ${SG_CFG:-r128x128x} --splits ${SG_SPLITS:-1,2,3} --json gpurun_out/sg_r.json
