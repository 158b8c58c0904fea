#!/bin/bash
# Round 5: the whole GPU suite and smoke(); cnn_op_info's tests and tables (comparator timing as the
# comparator's); VGG-19 b20 forwards reporting the resident filter-pack bytes (packs of the banks each
# route reads vs every Winograd bank)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
F=boda-1_amd/bin/boda_hip_rtc_fwd
tools/gpu_job.sh \
  gputests 800 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread -rf :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  vggpack 200 $F --net tests/golden/nets/vgg_19.prototxt --img 20 --iters 2 :: \
  vggpackall 200 $F --net tests/golden/nets/vgg_19.prototxt --img 20 --iters 2 --mode-args "(pack_all_banks=1)"
tools/job_cnn_op_info.sh
