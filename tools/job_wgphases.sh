#!/bin/bash
# Round 5: per-phase clocks (instrumented library) of the table's wgi routes in the conv set
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp BH_LIB_NAME=libboda_hip_ktrace.so
run() { timeout -k 10 120 python -u tools/wg_phases.py --conv "$1" --cfg "$2" --splits "$3" --slowest 12 >> gpurun_out/wgphases.log 2>&1 || exit $?; }
: > gpurun_out/wgphases.log
run 20,384,13,13,384,3,3,1,1,1,1 wgi128x32 11
run 20,256,13,13,384,3,3,1,1,1,1 wgi128x32 1
run 20,128,28,28,192,3,3,1,1,1,1 wgi128x32v 5
run 20,384,6,6,1024,3,3,1,1,1,1 wgi128x32 11
run 20,96,28,28,128,3,3,1,1,1,1 wgi128x32v 11
run 5,64,56,56,192,3,3,1,1,1,1 wgi128x32v 5
cat gpurun_out/wgphases.log
