#!/bin/bash
# Where the batch-20 1x1 ops' time goes: per-block device-clock marks (instrumented library) of their
# table routes, single calls (tools/ktrace.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=()
for s in "20 384 13 13 384 1 1 1 1 0 0" "20 512 14 14 144 1 1 1 1 0 0" "20 96 54 54 96 1 1 1 1 0 0" \
         "20 256 27 27 256 1 1 1 1 0 0" "20 1024 6 6 1000 1 1 1 1 0 0" "20 64 56 56 64 1 1 1 1 0 0"; do K+=(--conv "$s"); done
tools/gpu_job.sh ktrace1x1 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py "${K[@]}"
