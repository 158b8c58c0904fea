#!/bin/bash
# Closing validation of the final tree: full GPU suite, smoke, bench, b20 nets, rocprofv3 stats.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=tests/golden/nets
B=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 400 python -u bench.py --per-op gpurun_out/perop.json :: \
  alex20g 120 $B --net $N/alexnet_ng_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  nin20g 120 $B --net $N/nin_imagenet.prototxt --img 20 --iters 5 --graph 20 :: \
  gn20g 120 $B --net $N/googlenet_conv.prototxt --img 20 --iters 5 --graph 20 :: \
  res20g 120 $B --net $N/resnet-50.prototxt --img 20 --iters 5 --graph 20 :: \
  vgg20g 120 $B --net $N/vgg_19.prototxt --img 20 --iters 5 --graph 20 :: \
  profbench 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --eager --op-timing events --steps 3 --warmup 1 --no-cpu-baseline
