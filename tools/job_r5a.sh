#!/bin/bash
# Round 5: ABI-3 packs and the Winograd gate on GPU; element accuracy of direct routes on the 3x3
# list; retune of the op_sigs entries outside the gate (into a copy of the table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
tools/gpu_job.sh \
  tests 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_wgx.py tests/test_gpu_net.py -q --timeout 300 --timeout-method thread :: \
  acc 600 python -u tools/wino_gate.py --ops-file tools/ops_ops-prof-conv-3x3-cudnn-boda.txt --any \
    --force 128x128x32:0,128x128x32:4,128x128x32:8,128x128x32:-8,dm3w16x64c8:0,r128x128x32d2:0,gvs64x32w8:0 :: \
  tune 600 python -u tools/tune.py --sets op-sigs --key-re '^conv 1 (256 122 122 384 3 3|96 128 128 256 5 5) ' \
    --merge --keep-prev --confirm 3 --min-gain 0.02 --out gpurun_out/tune.out --json gpurun_out/tune_r5a.json
