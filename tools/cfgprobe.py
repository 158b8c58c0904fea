#!/usr/bin/env python3
"""Time chosen tile configurations x K-splits on a few shapes (graph-amortized, as the
bench's per-op time), next to the current tuned choice.

  python tools/cfgprobe.py --conv 20,64,56,56,192,3,3,1,1,1,1 --cfg r128 --splits 1,2
  python tools/cfgprobe.py --top 12 --cfg r      # the 12 conv ops with most roofline loss
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402
import tune  # noqa: E402

# "tuned" = the committed table's route (as in the bench), unless --no-table
_TABLE = os.path.join(ROOT, "boda-1_amd", "tuning", "gfx950.tune")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv", action="append", default=[])
    ap.add_argument("--sgemm", action="append", default=[])
    ap.add_argument("--top", type=int, default=0, help="take the N conv ops with the largest loss in --perop")
    ap.add_argument("--perop", default=os.path.join(ROOT, "profiles", "r01", "bench_perop.json"))
    ap.add_argument("--cfg", action="append", default=[], help="config-name prefix filter (repeatable; default r)")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--json", default="")
    ap.add_argument("--no-table", action="store_true", help="compare against the untuned heuristic")
    a = ap.parse_args()
    os.environ["BH_TUNE_FILE"] = "/nonexistent" if a.no_table else _TABLE
    shapes = [ops.ConvShape(*map(int, c.split(","))) for c in a.conv]
    shapes += [ops.SgemmShape(*map(int, c.split(","))) for c in a.sgemm]
    if a.top:
        d = [x for x in json.load(open(a.perop)) if x["tag"] == "conv"]
        d.sort(key=lambda x: -(x["kernel_ms"] * (1 - x["roofline_frac"])))
        shapes += [ops.ConvShape(*x["dims"]) for x in d[:a.top]]
    dev = boda_hip.Device(0)
    out = []
    for s in shapes:
        kind = 0 if isinstance(s, ops.SgemmShape) else 1
        wl = runner.Workload(dev, [s])
        dev.tune_set(kind, -1, 0)
        tune.time_op(dev, wl, 0, 3)  # (the first timing of a process runs ~10 % slow: clocks, caches)
        t0 = tune.time_op(dev, wl, 0, 3)
        rf = runner.roofline_secs(s) * 1e3
        print("%s  tuned %.4f ms (%.0f%% roofline)" % (s, t0, 100 * rf / t0), flush=True)
        for ci, cn in enumerate(boda_hip.tune_cfg_names(kind)):
            if not cn.startswith(tuple(a.cfg or ["r"])):
                continue
            for S in map(int, a.splits.split(",")):
                dev.tune_set(kind, ci, S)
                try:
                    t = tune.time_op(dev, wl, 0, 3)
                except boda_hip.UnsupportedError as e:
                    print("   %-16s S=%+d unsupported: %s" % (cn, S, e))
                    continue
                out.append({"shape": str(s), "cfg": cn, "splits": S, "ms": t, "tuned_ms": t0})
                print("   %-16s S=%+d %.4f ms (%.0f%% roofline)%s" % (cn, S, t, 100 * rf / t,
                                                                   "  <-- faster" if t < t0 else ""), flush=True)
        dev.tune_set(kind, -1, 0)
        wl.free()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=0)
    dev.close()


if __name__ == "__main__":
    main()
