#!/usr/bin/env python3
"""Record the dominant kernel's average launch duration from a rocprofv3 --kernel-trace --stats
summary (the *_kernel_stats.csv of the graph-replayed bench step), for bench.py's
roofline.frac_rocprof.

  python tools/rocprof_dominant.py profiles/r05/rocprof_graph_kernel_stats.csv \
      mfma32_sgemm_r128x128x32d2_vec_splitk_inkernel "ring_kernel<2, 2, 32, 2, 0, 2, 2>" \
      > profiles/rocprof_dominant.json

kernel: the bench line's roofline.kernel (variant name); symbol: the substring of the profiled
kernel's demangled name that identifies that variant's template instance.
"""
import csv
import json
import sys


def main():
    path, kernel, symbol = sys.argv[1:4]
    rows = [r for r in csv.DictReader(open(path)) if symbol in r["Name"]]
    if len(rows) != 1:
        sys.exit("expected one kernel matching %r, found %d" % (symbol, len(rows)))
    r = rows[0]
    json.dump({"kernel": kernel, "symbol": r["Name"], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
               "source": "rocprofv3 --kernel-trace --stats of the graph-replayed bench step: " + path},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
