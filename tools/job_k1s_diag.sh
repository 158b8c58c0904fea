#!/bin/bash
# k1s cost decomposition: diagnostic builds (instrumented library) + PMC passes on the plain kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_job.sh \
  diag 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 --conv 20,64,56,56,64,1,1,1,1,0,0 --cfg xks --splits 1,2 :: \
  diag2 300 env BH_LIB_NAME=libboda_hip_ktrace.so python -u tools/cfgprobe.py --conv 20,96,54,54,96,1,1,1,1,0,0 --conv 20,64,56,56,64,1,1,1,1,0,0 --cfg ks96c32q3 --splits 1,2 :: \
  pmc 500 tools/job_pmc_k1s.sh
