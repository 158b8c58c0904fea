#!/bin/bash
# Tune the nets' conv / fc shapes at b1 and b5 the table lacks, then the GPU suite and the
# nets at b1 / b5 with the merged table.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  tune 700 python -u tools/tune.py --sets nets-b1,nets-b5 --only-untuned --merge --out gpurun_out/gfx950.tune --json gpurun_out/tune_nets_b1b5.json :: \
  gputests 600 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  res1 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/resnet-50.prototxt --img 1 --iters 3 --graph 20 :: \
  vgg1 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/vgg_19.prototxt --img 1 --iters 3 --graph 20 :: \
  res5 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/resnet-50.prototxt --img 5 --iters 3 --graph 20 :: \
  vgg5 120 env BH_TUNE_FILE=gpurun_out/gfx950.tune $B --net $N/vgg_19.prototxt --img 5 --iters 3 --graph 20
