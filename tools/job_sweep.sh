#!/bin/bash
# full re-sweep (every config x split) of the conv-set ops matching KEY_RE into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/sweep.tune
tools/gpu_job.sh \
  tune 1100 python -u tools/tune.py --sets ${SETS:-conv} --key-re "$KEY_RE" --merge --out gpurun_out/sweep.tune --json gpurun_out/sweep_tune.json
