#!/bin/bash
# Round 5: the pixels-on-N resident-bank 1x1 kernel (kn*): parity of every ks / kn config (and the
# Winograd / ops-prof / direct suites after the F(4x4,3x3) IC cap), then every kn config timed on the
# 1x1 ops of the conv set and op_sigs next to the table's route, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=()
for s in 20,64,56,56,64 20,96,54,54,96 20,192,28,28,96 20,256,28,28,128 20,256,27,27,256 20,192,28,28,64 \
         20,256,28,28,64 20,256,28,28,32 20,192,28,28,32 20,192,28,28,16 20,528,14,14,160 20,512,14,14,144 \
         20,480,14,14,192 20,528,14,14,256 20,384,13,13,384 20,512,14,14,128 20,528,14,14,128 20,480,14,14,96 \
         5,96,54,54,96 5,64,56,56,64 5,256,27,27,256 5,192,28,28,96 5,256,28,28,128 5,128,56,56,128 \
         1,64,56,56,64 1,96,54,54,96 20,128,56,56,128 20,96,107,107,96 3,96,107,107,96; do
  P+=(--conv "$s,1,1,1,1,0,0")
done
tools/gpu_job.sh \
  tests 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_k1s.py tests/test_gpu_wgx.py \
    tests/test_gpu_opsprof.py tests/test_gpu_direct.py tests/test_gpu_configs.py -rf :: \
  knprobe 900 python -u tools/cfgprobe.py "${P[@]}" --cfg kn --splits 1,2 --json gpurun_out/probe_kn.json
