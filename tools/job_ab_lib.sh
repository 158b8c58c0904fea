#!/bin/bash
# Same-box A/B of two builds of the library (BH_LIB_NAME), alternating: the CFG configs (default wg)
# on conv-set shapes (AB_OPS: full dims, or WG_OPS: 3x3 s1 p1 shapes). AB_LIB = the variant library's
# file name under boda-1_amd/lib.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=()
if [ -n "${AB_OPS:-}" ]; then
  for d in $AB_OPS; do OPS+=(--conv "$d"); done
else
  for d in ${WG_OPS:-20,64,56,56,192 20,384,13,13,384 20,144,14,14,288 20,128,28,28,192 20,256,56,56,256}; do
    OPS+=(--conv "$d,3,3,1,1,1,1")
  done
fi
tools/gpu_job.sh \
  a1 200 env BH_LIB_NAME=${AB_BASE:-libboda_hip.so} python -u tools/cfgprobe.py "${OPS[@]}" --cfg ${CFG:-wg} --splits ${SPLITS:-11,15} --json gpurun_out/ab_a1.json :: \
  b1 200 env BH_LIB_NAME=$AB_LIB python -u tools/cfgprobe.py "${OPS[@]}" --cfg ${CFG:-wg} --splits ${SPLITS:-11,15} --json gpurun_out/ab_b1.json :: \
  a2 200 env BH_LIB_NAME=${AB_BASE:-libboda_hip.so} python -u tools/cfgprobe.py "${OPS[@]}" --cfg ${CFG:-wg} --splits ${SPLITS:-11,15} --json gpurun_out/ab_a2.json :: \
  b2 200 env BH_LIB_NAME=$AB_LIB python -u tools/cfgprobe.py "${OPS[@]}" --cfg ${CFG:-wg} --splits ${SPLITS:-11,15} --json gpurun_out/ab_b2.json
