#!/bin/bash
# net tests through has_conv_fwd_t (+ per-blob parity), dropout / layers, then ktrace of the k1s kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_job.sh \
  net 900 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_layers.py -x -v --timeout 900 --timeout-method thread :: \
  kt 200 python -u tools/ktrace.py --conv "20 96 54 54 96 1 1 1 1 0 0" --conv "20 192 28 28 32 1 1 1 1 0 0" --cfg ks96c32q3 --reps 3 :: \
  kt2 200 python -u tools/ktrace.py --conv "20 192 28 28 32 1 1 1 1 0 0" --conv "20 64 56 56 64 1 1 1 1 0 0" --cfg ks32c16q4 --reps 3
