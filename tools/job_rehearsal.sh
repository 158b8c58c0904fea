#!/bin/bash
# The multi-rank bench path on one leased GPU: 2 ranks (torch.distributed, RCCL), sharing the device
# (--rehearsal: "shared_device": true); the 1 -> 8 curve itself is the driver's, on an 8-GPU node
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --rehearsal --no-cpu-baseline --vendor off \
  > gpurun_out/rehearsal.log 2>&1; rc=$?
grep '"metric"' gpurun_out/rehearsal.log | tail -1 > gpurun_out/rehearsal_line.json
tail -3 gpurun_out/rehearsal.log | cut -c1-300
exit $rc
