#!/bin/bash
# Net executor rewrites (BatchNorm/Scale folding, in-place Concat slabs): GPU tests, then the
# batch-20 net forwards with and without them.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/nets
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  slabtests 300 python -u -m pytest tests/test_gpu_conv.py -k slab tests/test_gpu_net.py -x -v --timeout 120 --timeout-method thread :: \
  res20 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 :: \
  res20nf 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --no-fold :: \
  gn20 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 :: \
  gn20nc 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --no-inplace-concat :: \
  alex20 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 :: \
  vgg20 120 $B --net $N/vgg_19.prototxt --img 20 --iters 5
