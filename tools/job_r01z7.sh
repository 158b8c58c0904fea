#!/bin/bash
# Multi-process rehearsal of the driver's N>1 bench launch on the 1-GPU box (2 ranks share
# GPU 0): weak (default) and strong (--strong, LPT-sharded op list).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  bench2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline :: \
  bench2s 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --strong
