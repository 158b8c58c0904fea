cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/lat_bench > gpurun_out/lat_bench.log 2>&1 || exit $?
for s in "1 160 7 7 320 3 3 1 1 1 1" "5 832 7 7 48 1 1 1 1 0 0" "1 4096 1 1 1000 1 1 1 1 0 0" "20 832 7 7 256 1 1 1 1 0 0" "1 384 13 13 256 3 3 1 1 1 1" "20 528 14 14 128 1 1 1 1 0 0"; do
  timeout -k 10 60 python tools/ktrace.py --conv "$s" --reps 4 >> gpurun_out/kt1.log 2>&1 || exit $?
done
