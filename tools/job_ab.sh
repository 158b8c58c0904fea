#!/bin/bash
# A/B of two builds of libboda_hip on the table's routes of chosen ops (graph-amortized, as the
# bench): BH_LIB_NAME=$LIB_B vs the default library, alternated twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OPS=(); while read -r l; do OPS+=(--conv "$l"); done < "${OPS_FILE:-tools/ab_ops.txt}"
for r in 1 2; do
  echo "### default (round $r)" >> gpurun_out/ab.log
  timeout -k 10 200 python tools/cmpcfg.py "${OPS[@]}" --cand table >> gpurun_out/ab.log 2>&1 || exit $?
  echo "### $LIB_B (round $r)" >> gpurun_out/ab.log
  BH_LIB_NAME=$LIB_B timeout -k 10 200 python tools/cmpcfg.py "${OPS[@]}" --cand table >> gpurun_out/ab.log 2>&1 || exit $?
done
