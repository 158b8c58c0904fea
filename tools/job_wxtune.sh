#!/bin/bash
# Position-split Winograd: parity, a tuning pass of the wx* configs over the stride-1 3x3 / 5x5 ops of
# SETS against the table's choices (into a copy of the table), then the quick bench on that copy;
# PMC passes of the k1s kernel and one wx kernel through their table routes
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
    --no-cpu-baseline --per-op gpurun_out/perop_wx.json :: \
  pmck1s 400 tools/pmc.sh gpurun_out/pmck1s python3 tools/profile_op.py conv 20,96,54,54,96,1,1,1,1,0,0 --iters 20 :: \
  pmcwx 400 env BH_TUNE_FILE=gpurun_out/tune.out tools/pmc.sh gpurun_out/pmcwx python3 tools/profile_op.py conv 20,64,56,56,192,3,3,1,1,1,1 --iters 20
