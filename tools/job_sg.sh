#!/bin/bash
# big-SGEMM route probe: ring vs stream-K ring, splits, at the dominant kernel's sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_job.sh \
  sg 900 python -u tools/cfgprobe.py --sgemm 6144,6144,6144 --sgemm 10240,10240,10240 --sgemm 12288,12288,12288 --cfg srk128 --splits 1,2,5,6 :: \
  sg2 900 python -u tools/cfgprobe.py --sgemm 6144,6144,6144 --sgemm 10240,10240,10240 --cfg r128x128x32 --splits 1,2
