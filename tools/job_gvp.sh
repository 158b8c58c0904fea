#!/bin/bash
# gvp kernels: parity on GPU, then a gvp-only tuning pass over the conv set into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gvp.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_configs.py -k gvp -x -q --timeout 120 --timeout-method thread :: \
  tune 800 python -u tools/tune.py --sets conv --cfg-re '^gvp' --merge --out gpurun_out/gvp.tune --json gpurun_out/gvp_tune.json
