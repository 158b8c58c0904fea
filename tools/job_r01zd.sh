#!/bin/bash
# C4: tune the full nets' conv / fc shapes the table lacks (ResNet-50, VGG-19 at b20), then
# the b20 forwards with the merged table.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  tune 900 python -u tools/tune.py --sets nets --only-untuned --merge --out gpurun_out/gfx950.tune --json gpurun_out/tune_nets.json :: \
  res20t 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 :: \
  vgg20t 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/vgg_19.prototxt --img 20 --iters 5 --graph 20 :: \
  gn20t 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --graph 20
