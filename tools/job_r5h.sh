#!/bin/bash
# Round 5: retunes on one box into a copy of the table -- the 1x1 ops of conv + op_sigs against the
# resident-bank configs (ks / kn, every grid mode), the IC = 3 stems against every direct config
# (resident-weight dcr included), the mid-size 3x3 ops against the Winograd / dm configs; then the
# quick bench of conv + op_sigs on the result
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
T="python -u tools/tune.py --sets conv,op-sigs --merge --confirm 3 --min-gain 0.02 --out gpurun_out/tune.out"
tools/gpu_job.sh \
  t1x1 900 $T --key-re '^conv \d+ \d+ \d+ \d+ \d+ 1 1 1 1 0 0$' --cfg-re '^k[sn]' --json gpurun_out/tune_1x1.json :: \
  tstem 400 $T --key-re '^conv \d+ 3 ' --cfg-re '^dc' --json gpurun_out/tune_stem.json :: \
  t3x3 600 $T --key-re '^conv (20|5) \d+ (13 13|14 14|7 7|28 28) \d+ 3 3 1 1 1 1$' --cfg-re '^(w|dm)' --json gpurun_out/tune_3x3.json :: \
  bench 300 env BH_TUNE_FILE=gpurun_out/tune.out python -u bench.py --sets conv,op-sigs --steps 3 --warmup 1 \
    --vendor off --no-cpu-baseline --per-op gpurun_out/perop_rt.json
