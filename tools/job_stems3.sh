#!/bin/bash
# stems: parity of the dc configs, every dc config on the conv set's stems, PMC of the 11x11 s4 b20
# stem with the table's route and with the phase-split strip
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
P=()
for s in 20,3,224,224,64,7,7,2,2,3,3 20,3,227,227,96,11,11,4,4,0,0 20,3,224,224,96,11,11,4,4,0,0 \
         5,3,227,227,96,11,11,4,4,0,0 5,3,224,224,96,11,11,4,4,0,0 5,3,224,224,64,7,7,2,2,3,3 \
         1,3,227,227,96,11,11,4,4,0,0 1,3,224,224,96,11,11,4,4,0,0; do P+=(--conv "$s"); done
tools/gpu_job.sh \
  dctest 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_direct.py :: \
  stemprobe 600 python -u tools/cfgprobe.py "${P[@]}" --cfg dc --splits 0 --json gpurun_out/probe_dc.json :: \
  pmcst 400 tools/pmc.sh gpurun_out/pmcst python3 tools/profile_op.py conv 20,3,227,227,96,11,11,4,4,0,0 --iters 20 :: \
  pmcstp 400 tools/pmc.sh gpurun_out/pmcstp python3 tools/profile_op.py conv 20,3,227,227,96,11,11,4,4,0,0 --cfg dc11s4x32d2p --splits 0 --iters 20
