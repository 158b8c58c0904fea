#!/bin/bash
# diagnostic dcm builds (instrumented library): full vs no-DMA vs no-MFMA vs no-LDS-reads on one op
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BH_LIB_NAME=libboda_hip_ktrace.so timeout -k 10 200 python tools/cmpcfg.py --conv "20 384 13 13 384 3 3 1 1 1 1" \
  --cand dm3w16x128c8w8:2 --cand xdm3w16x128c8w8_nodma:2 --cand xdm3w16x128c8w8_nomfma:2 \
  --cand dm3w16x64c8:2 --cand xdm3w16x64c8_nodma:2 --cand xdm3w16x64c8_nomfma:2 --cand xdm3w16x64c8_none:2 \
  --cand xdm3w16x64c8_noread:2 --cand xdm3w16x64c8_nodma_noread:2 > gpurun_out/dbg.log 2>&1
