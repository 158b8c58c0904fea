#!/bin/bash
# parity on the conv kernels + quick per-op bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh \
  test 500 python -u -m pytest ${TESTS:-tests/test_gpu_direct.py tests/test_gpu_dcm.py tests/test_gpu_configs.py tests/test_gpu_conv.py tests/test_gpu_net.py} -x -q --timeout 120 --timeout-method thread :: \
  bench 400 python -u bench.py --sets ${SETS:-conv,op-sigs} --steps 3 --warmup 1 --vendor off --no-cpu-baseline --per-op gpurun_out/perop.json
