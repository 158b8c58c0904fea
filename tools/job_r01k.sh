#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  tests 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  cmp 300 python -u tools/cmpcfg.py --cand r64x128x32d3:1 --cand r128x128x16d4:1 --cand r128x64x32d3:1 --cand r64x256x32d3:1 --cand r128x128x32d2:1 --conv "20 3 224 224 64 7 7 2 2 3 3" --conv "20 3 227 227 96 11 11 4 4 0 0" --conv "5 3 224 224 64 7 7 2 2 3 3" :: \
  tune 1100 python -u tools/tune.py --sets conv --out gpurun_out/gfx950.tune --merge --json gpurun_out/tune_conv.json :: \
  bench 300 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u bench.py --per-op gpurun_out/perop.json
