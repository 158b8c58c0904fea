#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh test 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  probe 300 python -u tools/cfgprobe.py --conv 20,384,13,13,384,3,3,1,1,1,1 --conv 20,256,13,13,384,3,3,1,1,1,1 --conv 20,384,6,6,1024,3,3,1,1,1,1 --conv 20,144,14,14,288,3,3,1,1,1,1 --conv 20,160,7,7,320,3,3,1,1,1,1 --conv 20,192,7,7,384,3,3,1,1,1,1 --cfg wgp --splits 2,12
