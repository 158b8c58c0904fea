#!/bin/bash
# PMC comparison: the same GEMM (256 x 14580 x 2400) as conv 5x5 (ring, im2col B) and as SGEMM (ring, 16-B B)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  cmp 200 python -u tools/cmpcfg.py --cand r128x128x32d2:1 --cand r128x128x32d4:1 --conv "20 96 27 27 256 5 5 1 1 2 2" --sgemm "256 14580 2400" :: \
  pmcc 400 tools/pmc.sh gpurun_out/pmc_c5 python3 tools/profile_op.py conv 20,96,27,27,256,5,5,1,1,2,2 --cfg r128x128x32d4 --splits 1 --iters 10 :: \
  pmcs 400 tools/pmc.sh gpurun_out/pmc_s5 python3 tools/profile_op.py sgemm 256,14580,2400 --cfg r128x128x32d4 --splits 1 --iters 10
