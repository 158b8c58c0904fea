#!/bin/bash
# Round 5: the whole GPU suite (no -x: every failure listed), then every dc config timed on the
# conv set's stems next to the table's route, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=()
for s in 20,3,224,224,64,7,7,2,2,3,3 20,3,227,227,96,11,11,4,4,0,0 20,3,224,224,96,11,11,4,4,0,0 \
         5,3,227,227,96,11,11,4,4,0,0 5,3,224,224,96,11,11,4,4,0,0 5,3,224,224,64,7,7,2,2,3,3 \
         1,3,227,227,96,11,11,4,4,0,0 1,3,224,224,96,11,11,4,4,0,0 1,3,224,224,64,7,7,2,2,3,3; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  gputests 800 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf :: \
  stemprobe 600 python -u tools/cfgprobe.py "${P[@]}" --cfg dc --splits 0 --json gpurun_out/probe_dc.json
