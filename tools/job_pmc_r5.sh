#!/bin/bash
# Round 5 PMC records (tools/pmc.sh passes, tools/pmc_summary.py): the resident-bank 1x1 kernels
# (k1n on 20x96x54^2 -> 96, k1s on 20x64x56^2 -> 64) and the resident-weight stems (dcr on the b20
# 7x7 s2 and 11x11 s4 stems), each forced to the configuration named
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name dims cfg splits kernel
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc_$1 python3 tools/profile_op.py conv $2 --cfg $3 --splits $4 --iters 20 \
    || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 --kernel $5 --op "conv ${2//,/ } cfg=$3 splits=$4" \
    --json gpurun_out/pmc_$1.json || exit $?
}
run k1n 20,96,54,54,96,1,1,1,1,0,0 kn32p32c32q3w8 1 k1n_kernel
run k1s 20,96,54,54,96,1,1,1,1,0,0 ks32c32q3w8 2 k1s_kernel
run stem7 20,3,224,224,64,7,7,2,2,3,3 dc7s2r32d3v 0 dcr_kernel
run stem11 20,3,227,227,96,11,11,4,4,0,0 dc11s4r32d2 0 dcr_kernel
