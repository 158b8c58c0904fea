#!/bin/bash
# SGEMM: stream-K and ring configs on the big sgemm-ops-full shapes beside the table's route
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=()
for m in 10240 7168 6144 5120 3072 12288; do S+=(--sgemm "$m,$m,$m"); done
tools/gpu_job.sh \
  sgsrk 500 python -u tools/cfgprobe.py "${S[@]}" --cfg srk --splits 1,2,5,6 --json gpurun_out/sg_srk.json :: \
  sgr 600 python -u tools/cfgprobe.py "${S[@]}" --cfg r --splits 1,2,3,4 --json gpurun_out/sg_r.json
