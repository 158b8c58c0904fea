#!/bin/bash
# stems: every dc config on the conv set's stems, per-block marks of the table routes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=()
for s in 20,3,224,224,64,7,7,2,2,3,3 20,3,227,227,96,11,11,4,4,0,0 20,3,224,224,96,11,11,4,4,0,0 \
         5,3,227,227,96,11,11,4,4,0,0 5,3,224,224,64,7,7,2,2,3,3; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  stemprobe 300 python -u tools/cfgprobe.py "${P[@]}" --cfg dc --splits 0 --json gpurun_out/probe_dc.json :: \
  kt7 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 3 224 224 64 7 7 2 2 3 3" --cfg dc7s2x64n128d2v :: \
  kt11 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "20 3 227 227 96 11 11 4 4 0 0" --cfg dc11s4x32d2 :: \
  kt11b5 60 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/ktrace.py --conv "5 3 227 227 96 11 11 4 4 0 0" --cfg dc11s4x32d2
