#!/bin/bash
# A/B of a Winograd runtime switch on one box: the same probe with BH_WG_RD32=1 and =0, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
for d in 20,64,56,56,192 20,384,13,13,384 20,144,14,14,288 20,96,28,28,128 20,256,56,56,256; do
  OPS+=(--conv "$d,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  a1 200 env BH_WG_RD32=1 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits 11 --json gpurun_out/ab_a1.json :: \
  b1 200 env BH_WG_RD32=0 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits 11 --json gpurun_out/ab_b1.json :: \
  a2 200 env BH_WG_RD32=1 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits 11 --json gpurun_out/ab_a2.json :: \
  b2 200 env BH_WG_RD32=0 python -u tools/cfgprobe.py "${OPS[@]}" --cfg wg --splits 11 --json gpurun_out/ab_b2.json
