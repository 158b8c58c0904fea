#!/bin/bash
# dm kernel diagnostics (instrumented library): the production config beside its no-DMA /
# no-MFMA builds on one shape, amortized per-call time (tools/profile_op.py)
export BH_LIB_NAME=libboda_hip_ktrace.so
op=${1:-20,384,13,13,384,3,3,1,1,1,1}
for c in "dm3w16x64c8 3" "xdm3w16x64c8_nodma 3" "xdm3w16x64c8_nomfma 3" "xdm3w16x64c8_none 3" \
         "dm3w16x128c8w8 1" "xdm3w16x128c8w8_nodma 1" "xdm3w16x128c8w8_nomfma 1" \
         "xdm3w16x64c8_nodma_noread 3" "xdm3w16x64c8_noread 3"; do
  set -- $c
  timeout -k 10 60 python3 tools/profile_op.py conv $op --cfg $1 --splits $2 --iters 20 | grep median || exit 3
done
