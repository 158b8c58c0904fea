#!/bin/bash
# Round 5: re-sweep the Winograd configurations (grid modes incl. the combine-kernel ones) on the batch-20
# 3x3 / 5x5 stride-1 ops of the conv set and op_sigs (tuner: element gate, keep unless 2 % faster on
# medians of 3), then the table A B A B (A = tools/prev.tune, B = the re-swept table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
KEY_RE='conv 20 \d+ \d+ \d+ \d+ (3 3|5 5) 1 1' TUNE_ARGS='--cfg-re ^w[gx]' TUNE_SECS=900 tools/job_retune.sh && \
NEXT=gpurun_out/tune.out SETS=conv,op-sigs tools/job_ab_tab.sh
