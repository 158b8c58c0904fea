#!/bin/bash
# Winograd parity, a tuning pass of the wg* configs over the 3x3 stride-1 ops of SETS (into a copy
# of the table), then the quick bench on that copy (BH_TUNE_FILE)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets ${SETS:-conv,op-sigs} --cfg-re '^wg' --key-re '^conv \d+ \d+ \d+ \d+ \d+ 3 3 1 1 [01] [01]$' \
    --merge --out gpurun_out/tune.out --json gpurun_out/tune_wg.json :: \
  bench 400 env BH_TUNE_FILE=gpurun_out/tune.out python -u bench.py --sets conv,op-sigs --steps 3 --warmup 1 --vendor off \
    --no-cpu-baseline --per-op gpurun_out/perop_wg.json
