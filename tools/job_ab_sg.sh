#!/bin/bash
# sgemm-full quick bench, committed table vs the previous one (A B A B), same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then t=tools/prev.tune; else t=boda-1_amd/tuning/gfx950.tune; fi
    timeout -k 10 300 env BH_TUNE_FILE=$t python -u bench.py --sets sgemm-full --steps 3 --warmup 1 --vendor off \
      --no-cpu-baseline > gpurun_out/absg_${v}$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/absg_${v}$i.log').read().strip().splitlines()[-1]); print('$v$i', {k: (v['sum_kernel_ms'], v['roofline_frac']) for k, v in d['per_set'].items()})"
  done
done
