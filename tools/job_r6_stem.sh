#!/bin/bash
# Round 6: the resident-weight stem kernel with a phase-split strip (dcr *p configs): its tests, timings
# next to the table routes on the stem ops, and PMC (bank conflicts) of the new and the routed forms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_direct.py \
  -k "r32d2p or r32d3p or r64d2p or r64d3p" > gpurun_out/stem_tests.log 2>&1 || { tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -2 gpurun_out/stem_tests.log
args=""
for s in 20,3,227,227,96,11,11,4,4,0,0 5,3,227,227,96,11,11,4,4,0,0 20,3,224,224,96,11,11,4,4,0,0 \
         20,3,224,224,64,7,7,2,2,3,3 5,3,224,224,64,7,7,2,2,3,3 20,3,227,227,64,7,7,2,2,3,3; do
  args="$args --conv $s"
done
timeout -k 10 600 python -u tools/cfgprobe.py $args --cfg dc11s4r --cfg dc7s2r --cfg dc11s4x32d2 --cfg dc7s2x32d3 \
  --splits 0 --json gpurun_out/stem_probe.json > gpurun_out/stem_probe.log 2>&1 || { tail -30 gpurun_out/stem_probe.log; exit 1; }
grep -v unsupported gpurun_out/stem_probe.log
run() {  # name dims cfg kernel
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc_$1 python3 tools/profile_op.py conv $2 --cfg $3 --splits 0 --iters 20 \
    || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 --kernel $4 --op "conv ${2//,/ } cfg=$3 splits=0" \
    --json gpurun_out/pmc_$1.json || exit $?
}
run stem11p 20,3,227,227,96,11,11,4,4,0,0 dc11s4r32d2p dcr_kernel
run stem7p 20,3,224,224,64,7,7,2,2,3,3 dc7s2r32d3p dcr_kernel
run stem7 20,3,224,224,64,7,7,2,2,3,3 dc7s2r32d3v dcr_kernel
run stem11x 20,3,227,227,96,11,11,4,4,0,0 dc11s4x32d2 dc_kernel
