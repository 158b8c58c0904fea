#!/bin/bash
# PMC passes over one GoogLeNet b20 forward (pool / LRN / conv kernels per dispatch).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  pmcgn 400 tools/pmc.sh gpurun_out/pmc_gn boda-1_amd/bin/boda_hip_rtc_fwd --net tests/golden/nets/googlenet_conv.prototxt --img 20 --iters 1
