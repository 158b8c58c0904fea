#!/bin/bash
# Round 6: baseline bench line on this box, then PMC records of the Winograd routes the VERDICT asks
# for (wgi on 20x384x6^2->1024 and 20x256x13^2->384, wx43 on 20x64x56^2->192), each forced to its
# table route (tools/pmc.sh passes, tools/pmc_summary.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --per-op gpurun_out/bench_perop.json > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
run() {  # name dims cfg splits kernel
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc_$1 python3 tools/profile_op.py conv $2 --cfg $3 --splits $4 --iters 20 \
    || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 --kernel $5 --op "conv ${2//,/ } cfg=$3 splits=$4" \
    --json gpurun_out/pmc_$1.json || exit $?
}
run wgi6 20,384,6,6,1024,3,3,1,1,1,1 wgi128x32 31 wgp_kernel
run wgi13 20,256,13,13,384,3,3,1,1,1,1 wgi128x32 21 wgp_kernel
run wx43 20,64,56,56,192,3,3,1,1,1,1 wx43s10g 0 wgx_kernel
