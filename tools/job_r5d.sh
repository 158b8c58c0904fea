#!/bin/bash
# Round 5: ref64 known-good configuration, the config / direct / ops-prof GPU tests; retune of the
# stems with the resident-weight routes (into a copy of the table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
tools/gpu_job.sh \
  tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ref64.py tests/test_gpu_configs.py \
    tests/test_gpu_direct.py tests/test_gpu_opsprof.py -rf :: \
  tune 600 python -u tools/tune.py --sets conv,op-sigs --key-re '^conv \d+ 3 ' --merge --keep-prev --confirm 3 \
    --min-gain 0.02 --out gpurun_out/tune.out --json gpurun_out/tune_r5d.json
