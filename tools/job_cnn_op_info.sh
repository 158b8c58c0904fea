#!/bin/bash
# cnn_op_info on the GPU: its tests, then the conv-ops-1-5-20 and SGEMM eff tables against the
# rocBLAS / MIOpen comparator (eff rows: both sides in the reference's per-call event convention, the
# last of --run-iter calls; the graph-amortized per-call time of ours in the log), written under gpurun_out/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=boda-1_amd/bin/boda_hip_cnn_op_info
tools/gpu_job.sh \
  coitests 300 python -u -m pytest tests/test_cnn_op_info.py -x -v --timeout 120 --timeout-method thread :: \
  coiconv 600 $B --cnn-func-sigs-fn=tests/golden/ops/conv-ops-1-5-20-nin-alex-gn.txt --run-iter=5 --graph-reps=40 \
    --out-fn=gpurun_out/cnn_op_info_conv.txt --op-info-tab-fn=gpurun_out/conv_info_tab.tex \
    --op-eff-tab-fn=gpurun_out/conv_eff_tab.tex --eff-comp=1 --mrd-toler=3e-3 --show-mrd=1 :: \
  coiconvraw 600 $B --cnn-func-sigs-fn=tests/golden/ops/conv-ops-1-5-20-nin-alex-gn.txt --comp=none --run-iter=5 \
    --graph-reps=40 --print-format=1 --inc-op-info-in-eff=1 --op-eff-tab-fn=gpurun_out/conv_eff_tab.raw :: \
  coisgemm 300 $B --cnn-func-sigs-fn=tests/golden/ops/sgemm-ops-small.txt --run-iter=5 --graph-reps=10 \
    --out-fn=gpurun_out/cnn_op_info_sgemm.txt --op-info-tab-fn=gpurun_out/sgemm_info_tab.tex \
    --op-eff-tab-fn=gpurun_out/sgemm_eff_tab.tex --mrd-toler=2e-3
