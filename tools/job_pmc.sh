#!/bin/bash
# PMC passes (tools/pmc.sh) on chosen ops through their table routes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for d in ${PMC_OPS:-5,384,6,6,1024,3,3,1,1,1,1}; do
  i=$((i+1))
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc$i python3 tools/profile_op.py conv $d --iters 20 || exit $?
done
