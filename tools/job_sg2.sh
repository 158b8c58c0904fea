#!/bin/bash
# 256x128 8-wave ring: SGEMM config parity, then the big sizes against the current route
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_job.sh \
  test 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_policy.py -x -q --timeout 300 --timeout-method thread -k "sgemm_config or write_through" :: \
  sg 900 python -u tools/cfgprobe.py --sgemm 4096,4096,4096 --sgemm 6144,6144,6144 --sgemm 8192,8192,8192 --sgemm 10240,10240,10240 --sgemm 12288,12288,12288 --cfg r256 --splits 1
