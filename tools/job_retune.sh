#!/bin/bash
# Full-candidate retune of the table entries whose key matches KEY_RE (into a copy of the table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
tools/gpu_job.sh \
  tune ${TUNE_SECS:-1100} python -u tools/tune.py --sets ${SETS:-conv,op-sigs} --key-re "$KEY_RE" --merge \
    --out gpurun_out/tune.out --json gpurun_out/tune_retune.json
