#!/bin/bash
# Round close, part 1: the full GPU suite and smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  gputests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
