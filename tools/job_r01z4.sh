#!/bin/bash
# Forward-layer kernels (LRN channel chunks, pooling): layer + net tests, b20 net forwards.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  layertests 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread :: \
  alex20g 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  nin20g 120 $B --net $N/nin_imagenet.prototxt --img 20 --iters 5 --graph 20 :: \
  gn20g 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  res20g 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 :: \
  vgg20g 120 $B --net $N/vgg_19.prototxt --img 20 --iters 5 --graph 20
