#!/bin/bash
# Round 6: PMC of the lean-transform Winograd routes (wgl on the two ops of profiles/r06/pmc_wgi*.json), then
# a retune of the stem ops against every direct-conv config (dcr *p included) and a same-box A B A B of the
# committed table (A) against the result (B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name dims cfg splits kernel
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc_$1 python3 tools/profile_op.py conv $2 --cfg $3 --splits $4 --iters 20 \
    || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 --kernel $5 --op "conv ${2//,/ } cfg=$3 splits=$4" \
    --json gpurun_out/pmc_$1.json || exit $?
}
run wgl6 20,384,6,6,1024,3,3,1,1,1,1 wgl128x32 31 wgp_kernel
run wgl13 20,256,13,13,384,3,3,1,1,1,1 wgl128x32 31 wgp_kernel
KEY_RE='^conv [0-9]+ 3 22[47] 22[47] ' CFG_RE='^dc' MIN_GAIN=0.02 TUNE_SECS=600 PREV=boda-1_amd/tuning/gfx950.tune \
  bash tools/job_r6_retune.sh
