#!/bin/bash
# HBM traffic of bench.py's dominant kernel (roofline.traffic): run bench, list the
# shapes its dominant kernel ran, then one FETCH_SIZE and one WRITE_SIZE rocprofv3
# --pmc pass per shape (nothing else traced), and reduce to bytes per launch.
#   tools/traffic.sh <outdir> <dest json>
set -eu
out=$1; dest=$2
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --vendor off > "$out/bench.json"
python3 tools/traffic_shapes.py "$out/bench.json" > "$out/shapes.txt"
i=0
while read -r kind dims; do
  i=$((i+1)); d="$out/shape$i"; mkdir -p "$d"; echo "$kind $dims" > "$d/shape.txt"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$d/$ctr" -o pmc -- \
      python3 tools/profile_op.py "$kind" "$dims" --iters 2 > "$d/$ctr.log" 2>&1
  done
done < "$out/shapes.txt"
python3 tools/traffic_parse.py "$out" "$out/bench.json" "$dest"
