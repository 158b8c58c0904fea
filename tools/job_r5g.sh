#!/bin/bash
# Round 5: ops-prof multi-tune with the F(4x4,3x3) cap; ks / kn on the 1x1 ops with the one-unit-per-wave
# grid (S=8) next to the persistent grids; every Winograd / dm config on the mid-size 3x3 ops
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=()
for s in 20,64,56,56,64 20,96,54,54,96 20,192,28,28,96 20,256,28,28,128 20,256,27,27,256 20,192,28,28,64 \
         5,96,54,54,96 5,64,56,56,64 20,128,56,56,128 20,96,107,107,96; do
  P+=(--conv "$s,1,1,1,1,0,0")
done
Q=()
for s in 20,256,13,13,384 20,160,14,14,320 20,144,14,14,288 20,192,7,7,384 20,96,14,14,208 20,112,14,14,224 \
         20,128,14,14,256 20,160,7,7,320 5,384,13,13,384 5,256,13,13,384 5,128,28,28,192; do
  Q+=(--conv "$s,3,3,1,1,1,1")
done
tools/gpu_job.sh \
  tests 300 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_gpu_opsprof.py tests/test_gpu_k1s.py -rf :: \
  kprobe 600 python -u tools/cfgprobe.py "${P[@]}" --cfg k --splits 2,8 --json gpurun_out/probe_k8.json :: \
  wprobe 600 python -u tools/cfgprobe.py "${Q[@]}" --cfg w --splits 0,1,5,11,15 --json gpurun_out/probe_w.json
