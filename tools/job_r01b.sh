set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_job.sh \
  tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread :: \
  probe 400 python -u tools/cfgprobe.py --top 14 --cfg r --splits 1,2,3,4,6 --json gpurun_out/probe.json
