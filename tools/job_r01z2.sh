#!/bin/bash
# Net executor: GPU net tests, then batch-20 forwards with the whole-forward hipGraph timing.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  nettests 400 python -u -m pytest tests/test_gpu_net.py -x -v --timeout 120 --timeout-method thread :: \
  res20g 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 :: \
  gn20g 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  alex20g 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  nin20g 120 $B --net $N/nin_imagenet.prototxt --img 20 --iters 5 --graph 20 :: \
  vgg20g 120 $B --net $N/vgg_19.prototxt --img 20 --iters 5 --graph 20
