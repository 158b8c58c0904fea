#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=boda-1_amd/bin/boda_hip_rtc_fwd
N=tests/golden/nets
tools/gpu_job.sh \
  nettests 600 python -u -m pytest tests/test_gpu_net.py -x -v -s --timeout 300 --timeout-method thread :: \
  alex20 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 :: \
  gn20 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 :: \
  res20 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 :: \
  vgg20 120 $B --net $N/vgg_19.prototxt --img 20 --iters 5
