#!/bin/bash
# kernel traces of the small conv ops, replayed as the bench's per-op timing (tools/small_ops_trace.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_job.sh \
  sot1 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sot1 -o sot -- python3 tools/small_ops_trace.py --batch 1 --reps 40 --out gpurun_out/sot1_ops.json :: \
  sot5 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sot5 -o sot -- python3 tools/small_ops_trace.py --batch 5 --reps 40 --out gpurun_out/sot5_ops.json
