#!/bin/bash
# Round-1 measurement artifacts: rocprofv3 kernel stats of the bench command, HBM traffic of
# (rocprofv3 kernel tracing crashes inside hipGraphLaunch on this image: the profiled bench runs
# the same op list launched op by op, --eager --op-timing events)
# its dominant kernel (separate --pmc passes), ops-prof wisdom runs for wis-ana.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  profbench 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --eager --op-timing events --steps 3 --warmup 1 --no-cpu-baseline :: \
  opsprof 400 boda-1_amd/bin/boda_hip_ops_prof --ops-fn=tests/golden/ops/conv-ops-1-5-20-nin-alex-gn.txt --wisdom-in-fn=tests/golden/wis/conv-full-gen5.wis --wisdom-out-fn=gpurun_out/hip_conv.wis --write-runs=1 --run-iter=3 :: \
  traffic 500 tools/traffic.sh gpurun_out/traffic gpurun_out/traffic.json
