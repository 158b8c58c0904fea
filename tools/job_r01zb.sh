#!/bin/bash
# Full re-sweep of the conv set against the current kernels (every config; the table's
# choice is kept unless beaten by --min-gain), then the bench with the old and new tables.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  tune 1000 python -u tools/tune.py --sets conv --cfg-re . --merge --out gpurun_out/gfx950.tune --json gpurun_out/tune_conv_full.json :: \
  bench_old 300 python -u bench.py --no-cpu-baseline --per-op gpurun_out/perop_old.json :: \
  bench_new 300 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u bench.py --no-cpu-baseline --per-op gpurun_out/perop_new.json
