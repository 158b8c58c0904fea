#!/bin/bash
# quick bench for per-op data: conv + op-sigs sets, no vendor, no CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh \
  bench 400 python -u bench.py --sets ${SETS:-conv,op-sigs} --steps 3 --warmup 1 --vendor off --no-cpu-baseline --per-op gpurun_out/perop.json
