#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P="python -u tools/profile_op.py"
tools/gpu_job.sh \
  floor 120 python -u tools/floor.py --reps 100 :: \
  c1 60 $P conv 16,1024,32,32,1024,1,1,1,1,0,0 --cfg r128x128x32d4 --splits 1 :: \
  s1 60 $P sgemm 1024,16384,1024 --cfg r128x128x32d4 --splits 1 :: \
  c2 60 $P conv 16,1024,32,32,1024,1,1,1,1,0,0 --cfg 128x128x32 --splits 1 :: \
  s2 60 $P sgemm 1024,16384,1024 --cfg 128x128x16 --splits 1 :: \
  c3 60 $P conv 16,1024,34,34,1024,3,3,1,1,0,0 --cfg r128x128x32d4 --splits 1 :: \
  c4 60 $P conv 20,96,27,27,256,5,5,1,1,2,2 --cfg r128x128x32d4 --splits 1 :: \
  kt1 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "1 512 14 14 112 1 1 1 1 0 0" --conv "5 192 28 28 16 1 1 1 1 0 0" --conv "1 832 7 7 32 1 1 1 1 0 0" --conv "20 96 27 27 256 5 5 1 1 2 2"
