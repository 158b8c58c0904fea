#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  kt 120 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "1 512 14 14 64 1 1 1 1 0 0" --conv "20 512 4 4 128 1 1 1 1 0 0" --conv "1 832 7 7 48 1 1 1 1 0 0" --conv "5 512 14 14 128 1 1 1 1 0 0" :: \
  pmcstem 400 tools/pmc.sh gpurun_out/pmc_stem python3 tools/profile_op.py conv 20,3,224,224,64,7,7,2,2,3,3 --cfg r64x128x32d3 --splits 1 --iters 20
