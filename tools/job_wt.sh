#!/bin/bash
# policy tests + k1s retune (1x1 ops) + write-through pass over the conv and op_sigs tables
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_k1s.py -x -q --timeout 120 --timeout-method thread :: \
  tuneks 900 python -u tools/tune.py --sets conv,op-sigs --cfg-re '^ks' --key-re '^conv [0-9]+ [0-9]+ [0-9]+ [0-9]+ [0-9]+ 1 1 1 1 0 0' --merge --out gpurun_out/tune.out --json gpurun_out/tune_ks.json :: \
  tunewt 900 python -u tools/tune.py --sets conv,op-sigs --wt only --merge --out gpurun_out/tune.out --json gpurun_out/tune_wt.json
