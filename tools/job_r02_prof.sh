#!/bin/bash
# Round-2 measurement artifacts: HBM traffic of bench.py's dominant kernel (separate FETCH_SIZE /
# WRITE_SIZE --pmc passes), then rocprofv3 kernel stats of the bench's real graph-replayed step
# (round 1 recorded a crash of kernel tracing inside hipGraphLaunch; this is the rerun).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  traffic 600 tools/traffic.sh gpurun_out/traffic gpurun_out/traffic.json :: \
  profgraph 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_graph -o bench -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --vendor off
