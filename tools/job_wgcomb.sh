#!/bin/bash
# Round 5: the Winograd (wgp / wgi) cut-tile combine with double-buffered slab loads: parity, per-phase
# clocks, then a same-box A B A B of the conv set against the previous build (B = libboda_hip_prev.so:
# bh_wino.hip of the parent commit compiled into build/bh_wino_prev.o and linked with the other objects
# as boda-1_amd/Makefile links libboda_hip.so); profiles/r05/wg_combine/ab_shared_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_job.sh \
  wgtest 500 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_gpu_wino.py tests/test_gpu_configs.py -k "wg or streamk or repeatable" -rf && \
tools/job_wgphases.sh > gpurun_out/wgp_stdout.log 2>&1 && \
AB_ENV="BH_LIB_NAME=libboda_hip_prev.so" SETS=conv tools/job_ab_env.sh
