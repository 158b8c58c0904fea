#!/bin/bash
# Round 5: stream-K wx cut units summed by wx_combine_kernel (splits 20): wgx parity (bitwise equal to
# the last-arriver form), then a same-box table A B A B (A = profiles/r05/tables/prev.tune, B = with the splits-20 routes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh \
  wxtest 600 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_gpu_wgx.py tests/test_gpu_routed.py -rf && \
SETS=conv,op-sigs tools/job_ab_tab.sh
