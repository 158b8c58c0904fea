#!/usr/bin/env python3
"""Per-launch HBM bytes of the dominant kernel from separate FETCH_SIZE / WRITE_SIZE
rocprofv3 --pmc passes (tools/traffic.sh), corrected as MI355X_MICROARCH.md's HBM
section prescribes: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so it is doubled."""
import csv
import glob
import json
import os
import statistics
import sys

out_dir, bench_json, dest = sys.argv[1], sys.argv[2], sys.argv[3]
# the hot-path kernels (gen_data, stamps, runtime fills / copies, repacks and reduce passes excluded)
MAIN = ("gemm_kernel", "ring_kernel", "srk_kernel", "gv_kernel", "dc_kernel", "dcm_kernel")
b = json.loads([l for l in open(bench_json) if l.startswith("{")][-1])
per_shape = []
for d in sorted(glob.glob(os.path.join(out_dir, "shape*"))):
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(d, ctr, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        per = {}
        for r in csv.DictReader(open(f[0])):
            if not any(k in r["Kernel_Name"] for k in MAIN) or r["Counter_Name"] != ctr:
                continue
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        vals[ctr] = statistics.median(per.values()) if per else None
    if vals.get("FETCH_SIZE") is not None and vals.get("WRITE_SIZE") is not None:
        per_shape.append({"shape": open(os.path.join(d, "shape.txt")).read().strip(),
                          "fetch_kib": vals["FETCH_SIZE"], "write_kib": vals["WRITE_SIZE"],
                          "hbm_bytes": (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024})
res = {"kernel": b["roofline"]["kernel"],
       "bytes_per_launch": statistics.mean(x["hbm_bytes"] for x in per_shape) if per_shape else None,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on tools/profile_op.py per shape; "
                 "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB, median dispatch per shape, mean over shapes",
       "per_shape": per_shape}
json.dump(res, open(dest, "w"), indent=1)
print(json.dumps(res)[:400])
