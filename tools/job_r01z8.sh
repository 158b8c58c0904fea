#!/bin/bash
# A/B: the table's choice vs stream-K configs on the biggest conv ops.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
C="--conv '20 96 27 27 256 5 5 1 1 2 2' --conv '20 64 56 56 192 3 3 1 1 1 1' --conv '20 384 13 13 384 3 3 1 1 1 1' --conv '20 128 28 28 192 3 3 1 1 1 1'"
tools/gpu_job.sh \
  ab 300 bash -c "python -u tools/cmpcfg.py $C --cand table --cand srk128x128x32d2:1 --cand srk128x128x32d3:1 --cand srk128x128x32d4:1 --cand srk128x128x16d4:1 --cand srk128x128x32d2:2 --cand srk64x128x32d3:1 --cand srk64x128x32d3:2 --cand srk128x64x32d3:2 --cand srk64x256x32d3:1"
