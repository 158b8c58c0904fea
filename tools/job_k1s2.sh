#!/bin/bash
# k1s v2 parity + probe + ktrace; the new net / shard GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OPS=()
for d in 20,96,54,54,96 20,64,56,56,64 20,256,27,27,256 20,256,28,28,128 20,192,28,28,96 20,256,28,28,64 \
         20,192,28,28,64 20,192,28,28,32 20,384,13,13,384 20,480,14,14,192 20,512,14,14,160 20,832,7,7,384 \
         5,96,54,54,96 5,64,56,56,64 5,256,27,27,256 5,256,28,28,128 5,192,28,28,96 5,384,13,13,384; do
  OPS+=(--conv "$d,1,1,1,1,0,0")
done
tools/gpu_job.sh \
  test 400 python -u -m pytest tests/test_gpu_k1s.py -x -q --timeout 120 --timeout-method thread :: \
  probe 500 python -u tools/cfgprobe.py "${OPS[@]}" --cfg ks --splits 1,2 --json gpurun_out/k1s_probe.json :: \
  kt 200 python -u tools/ktrace.py --conv "20 96 54 54 96 1 1 1 1 0 0" --cfg ks96c32q3 --splits 1 --reps 3 :: \
  kt2 200 python -u tools/ktrace.py --conv "20 192 28 28 32 1 1 1 1 0 0" --conv "20 64 56 56 64 1 1 1 1 0 0" --cfg ks32c32q4 --reps 3 :: \
  net 900 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_shard.py -x -v --timeout 900 --timeout-method thread -k "dropout or mode_options or forward or panel or resnet or googlenet or unpacked"
