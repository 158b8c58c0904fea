#!/bin/bash
# k1s store policies + trace of the skeleton; PMC of the biggest-gap dcm op
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OPS=()
for d in 20,96,54,54,96 20,64,56,56,64 20,256,28,28,128 20,192,28,28,96 5,96,54,54,96 5,64,56,56,64; do
  OPS+=(--conv "$d,1,1,1,1,0,0")
done
tools/gpu_job.sh \
  probe 300 python -u tools/cfgprobe.py "${OPS[@]}" --cfg ks --splits 1,2 --json gpurun_out/k1s_probe2.json :: \
  kt 200 python -u tools/ktrace.py --conv "20 96 54 54 96 1 1 1 1 0 0" --cfg ks96c32q3w8 --splits 1 --reps 3 :: \
  kt2 200 python -u tools/ktrace.py --conv "20 96 54 54 96 1 1 1 1 0 0" --cfg xks96c32q3_none --splits 1 --reps 3 :: \
  pmc 500 tools/pmc.sh gpurun_out/pmcdm python3 tools/profile_op.py conv 20,64,56,56,192,3,3,1,1,1,1 --iters 20
