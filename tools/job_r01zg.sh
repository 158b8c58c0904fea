#!/bin/bash
# Final tree: smoke and bench as the driver runs them.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 400 python -u bench.py
