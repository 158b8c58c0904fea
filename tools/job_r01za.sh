#!/bin/bash
# C5 (op_sigs_full): tune the ops the table lacks, then the op-sigs bench with the old and the
# merged table.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/gfx950.tune
tools/gpu_job.sh \
  sigs_old 300 python -u bench.py --sets op-sigs --no-cpu-baseline --per-op gpurun_out/perop_sigs_old.json :: \
  tune 900 python -u tools/tune.py --sets op-sigs --only-untuned --merge --out gpurun_out/gfx950.tune --json gpurun_out/tune_sigs.json :: \
  sigs_new 300 env BH_TUNE_FILE=gpurun_out/gfx950.tune python -u bench.py --sets op-sigs --no-cpu-baseline --per-op gpurun_out/perop_sigs.json
