#!/bin/bash
# Round-1 final measurement set: full GPU tests, conv retune, bench, rocprofv3 kernel stats
# of the same bench command, HBM traffic of the dominant kernel (separate --pmc passes).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread :: \
  tune 1150 python -u tools/tune.py --sets conv --out gpurun_out/gfx950.tune --merge --json gpurun_out/tune_conv.json
