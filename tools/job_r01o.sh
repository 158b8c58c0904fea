#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C="--cand r128x128x32d2:1 --cand r128x128x32d2:2 --cand r64x128x32d3:1 --cand r128x64x32d3:1 --cand srk128x128x32d2:2 --cand srk128x128x16d4:2 --cand srk128x64x32d3:2 --cand srk64x128x32d3:2 --cand srk128x128x32d4:1 --cand srk64x64x32d4:2"
tools/gpu_job.sh \
  srktests 300 python -u -m pytest tests/test_gpu_configs.py -k "streamk" -x -q --timeout 120 --timeout-method thread :: \
  cmp 400 python -u tools/cmpcfg.py $C --conv "20 96 27 27 256 5 5 1 1 2 2" --conv "20 64 56 56 192 3 3 1 1 1 1" --conv "20 384 13 13 384 3 3 1 1 1 1" --conv "20 128 28 28 192 3 3 1 1 1 1" --conv "20 384 6 6 1024 3 3 1 1 1 1" --conv "20 144 14 14 288 3 3 1 1 1 1"
