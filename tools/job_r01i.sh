#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C="--cand table --cand r128x128x32d2:2 --cand r128x64x32d3:1 --cand r64x128x32d3:1 --cand srk128x128x32d2:2 --cand srk128x128x16d4:2 --cand srk128x64x32d3:2 --cand srk64x128x32d3:2 --cand srk128x128x32d4:1 --cand srk64x64x32d4:2"
tools/gpu_job.sh \
  newtests 300 python -u -m pytest tests/test_gpu_configs.py -k "streamk" -x -q --timeout 120 --timeout-method thread :: \
  cmp 300 python -u tools/cmpcfg.py $C --conv "20 96 27 27 256 5 5 1 1 2 2" --conv "20 64 56 56 192 3 3 1 1 1 1" --conv "20 384 13 13 384 3 3 1 1 1 1" --conv "20 144 14 14 288 3 3 1 1 1 1" --conv "5 384 13 13 256 3 3 1 1 1 1" --conv "20 3 224 224 64 7 7 2 2 3 3" --sgemm "2048 2048 2048"
