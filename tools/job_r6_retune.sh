#!/bin/bash
# Round 6: retune the conv set + op_sigs against new configs (CFG_RE, e.g. '^(kd|wgl)'), keeping each op's
# table route unless beaten by MIN_GAIN on medians of 3 re-timings (tools/job_retune.sh), then a same-box
# A B A B of the round's start table (A) against the result (B) in the bench's own per-op timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KEY_RE=${KEY_RE:-.} TUNE_ARGS="--cfg-re ${CFG_RE}" TUNE_SECS=${TUNE_SECS:-700} bash tools/job_retune.sh || exit $?
PREV=${PREV:-profiles/r06/tables/start.tune} NEXT=gpurun_out/tune.out bash tools/job_ab_tab.sh
