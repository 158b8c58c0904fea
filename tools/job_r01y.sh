#!/bin/bash
# Re-validation of HEAD on a fresh box: full GPU suite, smoke, bench, rocprofv3 kernel stats.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 400 python -u bench.py --per-op gpurun_out/perop.json :: \
  kstats 400 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1
