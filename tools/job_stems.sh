#!/bin/bash
# Direct stem configs: parity, then a tuning pass over the IC = 3 stems of conv + op_sigs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread :: \
  tune 600 python -u tools/tune.py --sets conv,op-sigs --key-re '^conv \d+ 3 ' --merge --out gpurun_out/tune.out --json gpurun_out/tune_stems.json
