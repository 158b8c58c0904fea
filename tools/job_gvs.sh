#!/bin/bash
# gvs kernels: parity, then a gvp/gvs tuning pass over the conv set into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gvs.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_configs.py -k "gvp or gv" -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets ${SETS:-conv} --cfg-re '^gv[ps]' --merge --out gpurun_out/gvs.tune --json gpurun_out/gvs_tune.json
