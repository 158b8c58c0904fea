#!/bin/bash
# PMC passes (tools/pmc.sh) of the k1s kernel on one op, forced config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 tools/pmc.sh gpurun_out/pmck1 python3 tools/profile_op.py conv ${OP:-20,96,54,54,96,1,1,1,1,0,0} --cfg ${CFG:-ks96c32q3} --splits ${SPL:-1} --iters 20
