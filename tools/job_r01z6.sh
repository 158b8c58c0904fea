#!/bin/bash
# Residual epilogue: C-ABI tests, net tests, ResNet-50 b20 forward.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  restests 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread :: \
  res20g 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 :: \
  res20nr 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 --no-resadd
