#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  srktests 300 python -u -m pytest tests/test_gpu_configs.py -k "streamk" -x -q --timeout 120 --timeout-method thread :: \
  tune 700 python -u tools/tune.py --sets conv --cfg-re "^srk" --out gpurun_out/gfx950.tune --merge --json gpurun_out/tune_srk.json :: \
  bench 300 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u bench.py --per-op gpurun_out/perop.json --no-cpu-baseline
