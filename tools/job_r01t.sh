#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  cfgtests 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread :: \
  cmp 200 python -u tools/cmpcfg.py --cand table --cand r128x128x32d2:1 --cand r128x128x32d4:1 --cand r64x128x32d3:1 --conv "20 96 27 27 256 5 5 1 1 2 2" --conv "20 64 56 56 192 3 3 1 1 1 1" --sgemm "256 14580 2400" :: \
  tune 900 python -u tools/tune.py --sets conv --out gpurun_out/gfx950.tune --merge --json gpurun_out/tune_conv.json :: \
  bench 300 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u bench.py --per-op gpurun_out/perop.json --no-cpu-baseline
