#!/bin/bash
# Same-box A B A B of two tuning tables in the bench's own per-op timing: A = $PREV (default profiles/r06/tables/start.tune),
# B = $NEXT (default the committed table); SETS (default conv,op-sigs); per-op files gpurun_out/abt_{A,B}{1,2}.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then t=${PREV:-profiles/r06/tables/start.tune}; else t=${NEXT:-boda-1_amd/tuning/gfx950.tune}; fi
    timeout -k 10 300 env BH_TUNE_FILE=$t python -u bench.py --sets ${SETS:-conv,op-sigs} --steps 3 --warmup 1 --vendor off \
      --no-cpu-baseline --per-op gpurun_out/abt_${v}$i.json > gpurun_out/abt_${v}$i.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abt_${v}$i.log').read().strip().splitlines()[-1]); print('$v$i', {k: (v['sum_kernel_ms'], v['roofline_frac']) for k, v in d['per_set'].items()})"
  done
done
