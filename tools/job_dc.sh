#!/bin/bash
# direct kernels (per-tile DMA planning, scalar channel offsets): parity, then a dc/dm-only
# retune of the conv set into a copy of the table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/dc.tune
tools/gpu_job.sh \
  test 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_dcm.py tests/test_gpu_configs.py -k "direct or dc or dm or gv" -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets conv --cfg-re '^d[cm]' --merge --out gpurun_out/dc.tune --json gpurun_out/dc_tune.json
