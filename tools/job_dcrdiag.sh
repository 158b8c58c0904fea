#!/bin/bash
# Diagnostic forms of the resident-weight stem kernel (instrumented library, wrong results by design):
# each drops one part of dc7s2r32d3v / dc11s4r32d2 on the b20 stems, to price it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BH_LIB_NAME=libboda_hip_ktrace.so timeout -k 10 300 python -u tools/cfgprobe.py --conv 20,3,224,224,64,7,7,2,2,3,3 \
  --cfg xdc7r --splits 0 --json gpurun_out/dcrdiag7.json > gpurun_out/dcrdiag7.log 2>&1 || exit $?
BH_LIB_NAME=libboda_hip_ktrace.so timeout -k 10 300 python -u tools/cfgprobe.py --conv 20,3,227,227,96,11,11,4,4,0,0 \
  --cfg xdc11r --splits 0 --json gpurun_out/dcrdiag11.json > gpurun_out/dcrdiag11.log 2>&1 || exit $?
BH_LIB_NAME=libboda_hip_ktrace.so timeout -k 10 300 python -u tools/cfgprobe.py --conv 20,3,224,224,64,7,7,2,2,3,3 \
  --conv 20,3,227,227,96,11,11,4,4,0,0 --cfg dc --splits 0 --json gpurun_out/dcrdiag_ref.json > gpurun_out/dcrdiag_ref.log 2>&1
