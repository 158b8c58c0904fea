#!/bin/bash
# GPU tests: TESTS = files, K = optional -k expression
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$K" ]; then
  tools/gpu_job.sh test 600 python -u -m pytest $TESTS -k "$K" -q --timeout 120 --timeout-method thread
else
  tools/gpu_job.sh test 600 python -u -m pytest $TESTS -q --timeout 120 --timeout-method thread
fi
