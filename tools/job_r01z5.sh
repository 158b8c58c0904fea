#!/bin/bash
# Round-1 closing measurement: full GPU suite, bench (default), rocprofv3 kernel stats of the
# same op list launched op by op (kernel tracing crashes inside hipGraphLaunch on this image).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 400 python -u bench.py --per-op gpurun_out/perop.json :: \
  profbench 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --eager --op-timing events --steps 3 --warmup 1 --no-cpu-baseline
