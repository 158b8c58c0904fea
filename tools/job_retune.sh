#!/bin/bash
# Full-candidate retune of the table entries whose key matches KEY_RE, on one box: the table's current
# choices are kept unless beaten by 2 % on medians of 3 re-timings of the top routes (tools/tune.py
# --keep-prev --confirm 3); the table is rewritten after every op, so a sweep cut short keeps its
# progress. BENCH=1: the quick bench on the result afterwards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp boda-1_amd/tuning/gfx950.tune gpurun_out/tune.out
export TMPDIR=/tmp
timeout -k 10 ${TUNE_SECS:-1000} python -u tools/tune.py --sets ${SETS:-conv,op-sigs} --key-re "$KEY_RE" --merge \
  --keep-prev --confirm 3 --min-gain ${MIN_GAIN:-0.02} ${TUNE_ARGS:-} --out gpurun_out/tune.out --json gpurun_out/tune_rt.json \
  > gpurun_out/tune_rt.log 2>&1
rc=$?
echo "tune rc=$rc"; tail -3 gpurun_out/tune_rt.log
[ $rc -eq 0 ] || [ $rc -eq 124 ] || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 env BH_TUNE_FILE=gpurun_out/tune.out python -u bench.py --sets conv,op-sigs --steps 3 --warmup 1 \
    --vendor off --no-cpu-baseline --per-op gpurun_out/perop_rt.json > gpurun_out/bench_rt.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_rt.log | cut -c1-300
fi
exit 0
