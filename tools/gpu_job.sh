#!/bin/bash
# Runs a list of GPU steps on the gpurun box, each under its own time limit.
# A step that exits 0 or 1 (e.g. a failing test) lets the job continue; a crash,
# abort, fault or timeout (anything else) ends the job immediately.
#   tools/gpu_job.sh <name> <seconds> <cmd...> [:: <name> <seconds> <cmd...>]...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
while [ $# -gt 0 ]; do
  name=$1; secs=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "::" ]; do cmd+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  echo "=== step $name (limit ${secs}s): ${cmd[*]}" | tee -a gpurun_out/job.log
  start=$(date +%s)
  timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/job.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc" | tee -a gpurun_out/job.log
    exit $rc
  fi
done
exit 0
