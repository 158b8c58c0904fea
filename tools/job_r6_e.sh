#!/bin/bash
# Round 6: the LDS-staged pooling kernel (tests + tools/layer_bench.py), and a check of which route the
# suite's 20x384x13^2->256 op takes in a fresh process
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "
import os, sys
sys.path.insert(0, 'boda-1_amd')
import boda_hip
print('table', os.path.exists('boda-1_amd/tuning/gfx950.tune'), boda_hip.LIB_PATH)
print('no ctx', boda_hip.variant_name(1, [20, 384, 13, 13, 256, 3, 3, 1, 1, 1, 1]))
d = boda_hip.Device(0)
print('ctx', d.variant(1, [20, 384, 13, 13, 256, 3, 3, 1, 1, 1, 1]))
" > gpurun_out/route_check.log 2>&1; cat gpurun_out/route_check.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layers.py \
  > gpurun_out/layers_tests.log 2>&1 || { tail -30 gpurun_out/layers_tests.log; exit 1; }
tail -2 gpurun_out/layers_tests.log
timeout -k 10 120 python -u tools/layer_bench.py --json gpurun_out/layer_bench2.json > gpurun_out/layer_bench2.log 2>&1
cat gpurun_out/layer_bench2.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py \
  > gpurun_out/conv_tests.log 2>&1; tail -5 gpurun_out/conv_tests.log
