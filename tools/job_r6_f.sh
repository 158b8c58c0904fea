#!/bin/bash
# Round 6: retune every stride-1 1x1 op of the conv set and op_sigs against the resident-bank 1x1 configs
# (ks / kn / kd / kw, the deep-ring ones included), then a same-box A B A B of the committed table (A)
# against the result (B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
KEY_RE=' 1 1 1 1 0 0$' CFG_RE='^k[sndw]' MIN_GAIN=0.02 TUNE_SECS=900 PREV=boda-1_amd/tuning/gfx950.tune \
  bash tools/job_r6_retune.sh
