#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  floor0 120 python -u tools/floor.py --reps 100 :: \
  floor1 120 env HIP_FORCE_DEV_KERNARG=1 python -u tools/floor.py --reps 100 :: \
  bench0 300 python -u bench.py --per-op gpurun_out/perop0.json --no-cpu-baseline :: \
  bench1 300 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py --per-op gpurun_out/perop1.json --no-cpu-baseline
