#!/bin/bash
# Round 5: the direct-stem kernels after the epilogue cut (biases start the accumulators, ReLU one
# v_max) and with deeper fragment prefetch (f<PF> configs): parity, then every dc config on the
# conv set's stems next to the table route, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=()
for s in 20,3,224,224,64,7,7,2,2,3,3 20,3,227,227,96,11,11,4,4,0,0 20,3,224,224,96,11,11,4,4,0,0 \
         5,3,227,227,96,11,11,4,4,0,0 5,3,224,224,96,11,11,4,4,0,0 5,3,224,224,64,7,7,2,2,3,3; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  dctest 600 python -u -m pytest -q --timeout 280 --timeout-method thread tests/test_gpu_direct.py tests/test_gpu_k1s.py -rf :: \
  stemprobe 600 python -u tools/cfgprobe.py "${P[@]}" --cfg dc --splits 0 --json gpurun_out/probe_dc2.json
