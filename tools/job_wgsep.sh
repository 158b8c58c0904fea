#!/bin/bash
# Round 5: stream-K Winograd cut tiles summed by a separate combine kernel (grid modes + 20): Winograd
# parity (every wg config and grid mode, the table's routes), per-phase clocks, then a same-box
# A B A B of the conv set and op_sigs, table without (A = profiles/r05/tables/prev.tune) and with (B) the + 20 routes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh \
  wgtest 600 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_routed.py tests/test_gpu_configs.py -k "wg or wino or streamk or repeatable or routed" -rf && \
SETS=conv,op-sigs tools/job_ab_tab.sh
