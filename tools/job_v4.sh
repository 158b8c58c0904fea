#!/bin/bash
# 16-B strip stems (dc*v) + gvo 1x1 kernels: parity, then a dc/gvo tuning pass into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/v4.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_configs.py -k "direct or gvo" -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets conv,op-sigs --cfg-re '^(dc|gvo)' --merge --out gpurun_out/v4.tune --json gpurun_out/v4_tune.json
