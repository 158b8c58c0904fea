#!/bin/bash
# Round 5: retune of the op_sigs 5x5 entry outside the Winograd gate (full-tensor gate), the ops-prof
# / routed / conv-set GPU tests on that table, the quick bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
tools/gpu_job.sh \
  tune 600 python -u tools/tune.py --sets op-sigs --key-re '^conv 1 96 128 128 256 5 5 ' \
    --merge --keep-prev --confirm 3 --min-gain 0.02 --out gpurun_out/tune.out --json gpurun_out/tune_r5b.json :: \
  tests 900 env BH_TUNE_FILE=gpurun_out/tune.out python -u -m pytest tests/test_gpu_opsprof.py tests/test_gpu_routed.py \
    tests/test_gpu_conv.py -q -rA --timeout 600 --timeout-method thread :: \
  bench 400 env BH_TUNE_FILE=gpurun_out/tune.out python -u bench.py --sets conv,op-sigs --steps 3 --warmup 1 --vendor off \
    --no-cpu-baseline --per-op gpurun_out/perop_r5b.json
