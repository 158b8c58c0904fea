#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 tools/kernarg_bench > gpurun_out/kb.log 2>&1 && timeout -k 10 120 tools/kernarg_bench >> gpurun_out/kb.log 2>&1; cat gpurun_out/kb.log
