#!/bin/bash
# Same-box A/B of an environment switch (AB_ENV, e.g. BH_PRIO=1): the quick bench on SETS, A B A B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in A B; do
    if [ $v = B ]; then e="env $AB_ENV"; else e=env; fi
    timeout -k 10 300 $e python -u bench.py --sets ${SETS:-conv,op-sigs} --steps 3 --warmup 1 --vendor off \
      --no-cpu-baseline --per-op gpurun_out/ab_${v}$i.json > gpurun_out/ab_${v}$i.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}$i.log').read().strip().splitlines()[-1]); print('$v$i', {k: (v['sum_kernel_ms'], v['roofline_frac']) for k, v in d['per_set'].items()})"
  done
done
