#!/bin/bash
# LRN / pooling kernel changes: layer tests, then the nets that use them.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  layertests 300 python -u -m pytest tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread :: \
  nettests 300 python -u -m pytest tests/test_gpu_net.py -x -q --timeout 120 --timeout-method thread -k "alexnet or googlenet" :: \
  alex20g 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  gn20g 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --graph 20
