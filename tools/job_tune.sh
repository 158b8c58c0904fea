#!/bin/bash
# Parity of a config family, then a tuning pass restricted to it, into a copy of the table
# (compare with the committed table, adopt by copying gpurun_out/tune.out over it):
#   CFG_RE='^gv[ps]' SETS=conv,op-sigs TESTS="tests/test_gpu_configs.py" K=gv tools/job_tune.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
tools/gpu_job.sh \
  test 600 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py} -k "${K:-gv}" -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets ${SETS:-conv} --cfg-re "$CFG_RE" --merge --out gpurun_out/tune.out --json gpurun_out/tune.json
