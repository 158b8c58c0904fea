#!/bin/bash
# Round close, part 3 (after a late kernel-source change): the GPU suite, smoke(), and the rocprofv3 kernel
# stats of the bench's graph-replayed step again, so that profiles/rocprof_dominant.json records this build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  gputests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  profgraph 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_graph -o bench -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --vendor off --op-timing events \
    --per-op gpurun_out/bench_perop_prof.json
