#!/bin/bash
# Round 6 GPU jobs, one step per call: bash tools/job_r6.sh <step> (outputs under gpurun_out/; the kept
# copies under profiles/r06/, cited in DESIGN.md). Steps:
#   pmc       baseline bench line, then PMC of the Winograd routes (wgi 20x384x6^2->1024 / 20x256x13^2->384,
#             wx43 20x64x56^2->192)                                   -> profiles/r06/pmc_{wgi6,wgi13,wx43}.json
#   kd        k1d (kd*) and lean-transform Winograd (wgl*) tests + probes, op-37 ops-prof log
#                                                                     -> probes/kd_probe_first.json, wgl_probe.json
#   kd2       k1d with a unit's whole input in flight + the no-store diagnostic builds
#                                                                     -> probes/kd_probe_deepring.json, kd_nostore_diag.log
#   nostore   k1n with the epilogue's stores dropped (instrumented library) next to the stored forms
#                                                                     -> probes/kn_nostore.log, kn_store.log
#   wgl       retune of the 3x3 stride-1 ops against wgl + same-box table A B A B -> ab/wgl_*
#   kw        store-wave k1w (kw*) tests + probes                     -> probes/kw_*
#   stem      phase-split dcr stems: tests, probes, PMC               -> stems/
#   deep      k1n / k1w with a unit's whole K in flight                -> probes/deep_*
#   wglpmc    PMC of the wgl routes, then the stem retune + A B A B  -> pmc_wgl{6,13}.json, ab/stem_*
#   pool      pooling tests + tools/layer_bench.py                    -> layers/
#   k1x1      retune of every 1x1 op against ks / kn / kd / kw + A B A B -> ab/k1x1_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"

pmcrun() {  # name dims cfg splits kernel
  timeout -k 10 400 tools/pmc.sh gpurun_out/pmc_$1 python3 tools/profile_op.py conv $2 --cfg $3 --splits $4 --iters 20 \
    || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_$1 --kernel $5 --op "conv ${2//,/ } cfg=$3 splits=$4" \
    --json gpurun_out/pmc_$1.json || exit $?
}
convs() {  # suffix shape...: --conv args
  local suf=$1 a=""
  shift
  for s in "$@"; do a="$a --conv $s$suf"; done
  echo "$a"
}
retune() {  # KEY_RE CFG_RE TUNE_SECS PREV
  KEY_RE="$1" CFG_RE="$2" MIN_GAIN=${MIN_GAIN:-0.02} TUNE_SECS=$3 PREV=$4 bash tools/job_r6_retune.sh
}
K1=,1,1,1,1,0,0
W3=,3,3,1,1,1,1

case "$1" in
pmc)
  timeout -k 10 400 python3 -u bench.py --per-op gpurun_out/bench_perop.json > gpurun_out/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
  pmcrun wgi6 20,384,6,6,1024,3,3,1,1,1,1 wgi128x32 31 wgp_kernel
  pmcrun wgi13 20,256,13,13,384,3,3,1,1,1,1 wgi128x32 21 wgp_kernel
  pmcrun wx43 20,64,56,56,192,3,3,1,1,1,1 wx43s10g 0 wgx_kernel
  ;;
kd)
  timeout -k 10 600 $T tests/test_gpu_k1s.py -k "kd" tests/test_gpu_nan.py > gpurun_out/kd_tests.log 2>&1 || exit 1
  timeout -k 10 600 $T tests/test_gpu_wino.py -k "wgl" > gpurun_out/wgl_tests.log 2>&1 || exit 1
  timeout -k 10 600 python -u tools/cfgprobe.py $(convs $K1 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 \
    20,192,28,28,96 20,256,28,28,128 20,256,28,28,64 20,192,28,28,64 20,192,28,28,32 20,256,28,28,32 20,192,28,28,16 \
    5,256,28,28,64 5,192,28,28,96) --cfg kd --splits 0,1,2,8 --json gpurun_out/kd_probe.json \
    > gpurun_out/kd_probe.log 2>&1 || exit 1
  timeout -k 10 900 python -u tools/cfgprobe.py $(convs $W3 20,384,13,13,384 20,256,13,13,384 20,128,28,28,192 \
    20,384,6,6,1024 5,64,56,56,192 20,96,28,28,128 20,144,14,14,288 20,160,14,14,320 20,128,14,14,256 20,112,14,14,224 \
    20,384,13,13,256) --cfg wg --splits 1,5,11,21,31 --json gpurun_out/wgl_probe.json > gpurun_out/wgl_probe.log 2>&1 \
    || exit 1
  timeout -k 10 700 bash tools/opsprof_op37.sh
  ;;
kd2)
  timeout -k 10 600 $T tests/test_gpu_k1s.py -k "kd" > gpurun_out/kd2_tests.log 2>&1 || exit 1
  timeout -k 10 600 python -u tools/cfgprobe.py $(convs $K1 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 \
    20,192,28,28,96 1,96,256,256,96) --cfg kd --splits 0,8 --json gpurun_out/kd2_probe.json \
    > gpurun_out/kd2_probe.log 2>&1 || exit 1
  timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py \
    $(convs $K1 20,96,54,54,96 5,96,54,54,96) --cfg xkd --splits 0 > gpurun_out/kd2_diag.log 2>&1
  ;;
nostore)
  A=$(convs $K1 20,96,54,54,96 1,96,256,256,96 20,64,57,57,64)
  timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py $A --cfg xkn --cfg xks \
    --splits 1,8 > gpurun_out/kn_nostore.log 2>&1 || exit 1
  timeout -k 10 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py $A --cfg kn32p32c32q3w8 \
    --cfg kn32p32c16q4w8 --cfg kn96p64c8q4w4 --cfg ks96c32q3 --splits 1,8 > gpurun_out/kn_store.log 2>&1
  ;;
wgl)
  MIN_GAIN=0.01 retune ' 3 3 1 1 [01] [01]$' '^wgl' 900 profiles/r06/tables/start.tune
  ;;
kw)
  timeout -k 10 600 $T tests/test_gpu_k1s.py tests/test_gpu_nan.py -k "kw" > gpurun_out/kw_tests.log 2>&1 || exit 1
  timeout -k 10 600 python -u tools/cfgprobe.py $(convs $K1 20,96,54,54,96 5,96,54,54,96 20,64,56,56,64 5,64,56,56,64 \
    20,64,57,57,64 20,192,28,28,96 1,96,256,256,96) --cfg kw --splits 1,2,8 --json gpurun_out/kw_probe.json \
    > gpurun_out/kw_probe.log 2>&1
  ;;
stem)
  timeout -k 10 600 $T tests/test_gpu_direct.py -k "r32d2p or r32d3p or r64d2p or r64d3p" > gpurun_out/stem_tests.log 2>&1 \
    || exit 1
  timeout -k 10 600 python -u tools/cfgprobe.py $(convs "" 20,3,227,227,96,11,11,4,4,0,0 5,3,227,227,96,11,11,4,4,0,0 \
    20,3,224,224,96,11,11,4,4,0,0 20,3,224,224,64,7,7,2,2,3,3 5,3,224,224,64,7,7,2,2,3,3 20,3,227,227,64,7,7,2,2,3,3) \
    --cfg dc11s4r --cfg dc7s2r --cfg dc11s4x32d2 --cfg dc7s2x32d3 --splits 0 --json gpurun_out/stem_probe.json \
    > gpurun_out/stem_probe.log 2>&1 || exit 1
  pmcrun stem11p 20,3,227,227,96,11,11,4,4,0,0 dc11s4r32d2p dcr_kernel
  pmcrun stem7p 20,3,224,224,64,7,7,2,2,3,3 dc7s2r32d3p dcr_kernel
  pmcrun stem7 20,3,224,224,64,7,7,2,2,3,3 dc7s2r32d3v dcr_kernel
  pmcrun stem11x 20,3,227,227,96,11,11,4,4,0,0 dc11s4x32d2 dc_kernel
  ;;
deep)
  timeout -k 10 600 $T tests/test_gpu_k1s.py -k "q12 or q6" > gpurun_out/deep_tests.log 2>&1 || exit 1
  timeout -k 10 600 python -u tools/cfgprobe.py $(convs $K1 20,96,54,54,96 5,96,54,54,96 20,192,28,28,96 1,96,256,256,96 \
    20,96,55,55,96) --cfg kn32p32c8q12 --cfg kn32p32c16q6 --cfg kw96c8q12 --cfg kw96c16q6 --cfg kw32c8q12 \
    --splits 1,2,8 --json gpurun_out/deep_probe.json > gpurun_out/deep_probe.log 2>&1
  ;;
wglpmc)
  pmcrun wgl6 20,384,6,6,1024,3,3,1,1,1,1 wgl128x32 31 wgp_kernel
  pmcrun wgl13 20,256,13,13,384,3,3,1,1,1,1 wgl128x32 31 wgp_kernel
  retune '^conv [0-9]+ 3 22[47] 22[47] ' '^dc' 600 boda-1_amd/tuning/gfx950.tune
  ;;
pool)
  timeout -k 10 300 $T tests/test_gpu_layers.py > gpurun_out/layers_tests.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/layer_bench.py --json gpurun_out/layer_bench.json > gpurun_out/layer_bench.log 2>&1
  ;;
k1x1)
  retune ' 1 1 1 1 0 0$' '^k[sndw]' 650 boda-1_amd/tuning/gfx950.tune
  ;;
*)
  echo "usage: bash tools/job_r6.sh {pmc|kd|kd2|nostore|wgl|kw|stem|deep|wglpmc|pool|k1x1}" >&2
  exit 2
  ;;
esac
