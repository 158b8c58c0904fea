#!/usr/bin/env python3
"""Record the dominant kernel's average launch duration from a rocprofv3 --kernel-trace --stats
summary (the *_kernel_stats.csv of the graph-replayed bench step), for bench.py's
roofline.frac_rocprof.

  python tools/rocprof_dominant.py profiles/r06/rocprof_graph_kernel_stats.csv \
      mfma32_sgemm_r128x128x32d2_vec_splitk_inkernel "ring_kernel<2, 2, 32, 2, 0, 2, 2>" \
      profiles/r06/bench_perop.json > profiles/rocprof_dominant.json

kernel: the bench line's roofline.kernel (variant name); symbol: the substring of the profiled
kernel's demangled name that identifies that variant's template instance; perop: the per-op file of
a bench run of the same build, whose units on that variant (their dims) are recorded with the build
hash (bench.build_hash: the kernel sources and the tuning table), so that bench.py reports
frac_rocprof only for the same launches of the same build.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    path, kernel, symbol, perop = sys.argv[1:5]
    from bench import build_hash
    rows = [r for r in csv.DictReader(open(path)) if symbol in r["Name"]]
    if len(rows) != 1:
        sys.exit("expected one kernel matching %r, found %d" % (symbol, len(rows)))
    r = rows[0]
    units = sorted(u["dims"] for u in json.load(open(perop)) if u["variant"] == kernel)
    if not units:
        sys.exit("no unit of %s in %s" % (kernel, perop))
    json.dump({"kernel": kernel, "symbol": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
               "units": units, "build_hash": build_hash(),
               "source": "rocprofv3 --kernel-trace --stats of the graph-replayed bench step: " + path},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
