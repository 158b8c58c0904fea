#!/bin/bash
# Position-split Winograd: parity, a tuning pass of the wx* configs over the stride-1 3x3 / 5x5 ops of
# SETS against the table's choices (into a copy of the table), then the quick bench on that copy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
tools/gpu_job.sh \
  test 600 python -u -m pytest tests/test_gpu_wgx.py -x -q --timeout 120 --timeout-method thread :: \
  tune 900 python -u tools/tune.py --sets ${SETS:-conv,op-sigs} --cfg-re '^wx' \
    --key-re '^conv \d+ \d+ \d+ \d+ \d+ (3 3 1 1 [01] [01]|5 5 1 1 [012] [012])$' \
    --merge --out gpurun_out/tune.out --json gpurun_out/tune_wx.json :: \
  bench 400 env BH_TUNE_FILE=gpurun_out/tune.out python -u bench.py --sets conv,op-sigs --steps 3 --warmup 1 --vendor off \
    --no-cpu-baseline --per-op gpurun_out/perop_wx.json
