#!/bin/bash
# remaining GPU suites + short-K 1x1 dcm configs: parity, then a dm1 tuning pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/dm1.tune
tools/gpu_job.sh \
  test 600 python -u -m pytest tests/test_gpu_opsprof.py tests/test_gpu_routed.py tests/test_gpu_rtc.py tests/test_gpu_sgemm.py tests/test_gpu_vendor.py tests/test_gpu_dcm.py -q --timeout 120 --timeout-method thread :: \
  tune 500 python -u tools/tune.py --sets conv,op-sigs --cfg-re '^dm1' --merge --out gpurun_out/dm1.tune --json gpurun_out/dm1_tune.json
