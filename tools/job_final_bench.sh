#!/bin/bash
# Round close, part 2: the default bench line (N=1), the dominant kernel's HBM traffic (separate
# FETCH_SIZE / WRITE_SIZE passes), rocprofv3 kernel stats of the bench's graph-replayed step (per-op
# timing by events: kernel tracing + the per-op graph pass crash the profiler,
# profiles/r02/rocprof_graph_crash.md)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  bench 600 python -u bench.py --per-op gpurun_out/bench_perop.json :: \
  traffic 600 tools/traffic.sh gpurun_out/traffic gpurun_out/traffic.json :: \
  profgraph 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_graph -o bench -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --vendor off --op-timing events
# then, here: the dominant kernel's rocprof average for bench.py's roofline.frac_rocprof
#   python tools/rocprof_dominant.py <the profgraph stats csv> <roofline.kernel> "<its template instance>" \
#     > profiles/rocprof_dominant.json
