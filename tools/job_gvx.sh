#!/bin/bash
# interleaved-column gv configs: parity, then a gv-family tuning pass over conv + op_sigs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gvx.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_configs.py -k "gv" -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets conv,op-sigs --cfg-re 'xw' --merge --out gpurun_out/gvx.tune --json gpurun_out/gvx_tune.json
