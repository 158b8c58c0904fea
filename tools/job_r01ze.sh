#!/bin/bash
# The conv heuristic (untuned shapes): GPU tests through it, and the nets with no table.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  vgg20h 120 env BH_TUNE_FILE=/nonexistent $B --net $N/vgg_19.prototxt --img 20 --iters 3 --graph 10 :: \
  res20h 120 env BH_TUNE_FILE=/nonexistent $B --net $N/resnet-50.prototxt --img 20 --iters 3 --graph 10 :: \
  gn20h 120 env BH_TUNE_FILE=/nonexistent $B --net $N/googlenet_conv.prototxt --img 20 --iters 3 --graph 10 :: \
  bench 300 python -u bench.py --no-cpu-baseline
