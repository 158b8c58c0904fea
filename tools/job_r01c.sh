#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  tests 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  bench 400 python -u bench.py --per-op gpurun_out/perop.json
