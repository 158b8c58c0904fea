#!/bin/bash
# 256-pixel dcm tiles: parity, then a dm-only tuning pass over the conv set into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/n256.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_dcm.py -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets conv,op-sigs --cfg-re '^dm' --merge --out gpurun_out/n256.tune --json gpurun_out/n256_tune.json
