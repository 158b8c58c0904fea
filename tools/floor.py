#!/usr/bin/env python3
"""Launch-floor probe: per-call GPU time of tiny calls, measured with the same
kernel-dispatch events ops-prof uses (bh_time_next_call) and, when run under
`rocprofv3 --kernel-trace --stats`, comparable with the profiler's durations.

  python tools/floor.py [--reps 200] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "boda-1_amd"))

import boda_hip as bh  # noqa: E402
from boda_hip.ops import ConvShape, SgemmShape  # noqa: E402
from boda_hip.runner import Workload  # noqa: E402


def timed(dev, fn, reps):
    ids = []
    for _ in range(reps):
        ids.append(dev.time_next_call())
        fn()
    dev.sync()
    us = [dev.elapsed_ms(b, e) * 1e3 for b, e in ids]
    dev.events_reset()
    return {"median_us": statistics.median(us), "min_us": min(us), "mean_us": statistics.fmean(us)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--json")
    ap.add_argument("--shapes", default="1 192 28 28 16 1 1 1 1 0 0;20 192 28 28 16 1 1 1 1 0 0;"
                                        "1 832 7 7 48 1 1 1 1 0 0;5 480 14 14 64 1 1 1 1 0 0")
    args = ap.parse_args()
    res = {}
    with bh.Device(0) as dev:
        tiny = dev.alloc_floats(64)
        res["gen_data_4"] = timed(dev, lambda: dev.gen_data(bh.GEN_CONV_BIASES, tiny, [4], 5), args.reps)
        # back-to-back floor inside a replayed graph: stamp kernels only (one lane each),
        # and tiny gen_data calls between stamps
        for label, body in (("graph: stamp->stamp", None),
                            ("graph: gen_data_4 between stamps", lambda: dev.gen_data(bh.GEN_CONV_BIASES, tiny, [4], 5))):
            n = 100
            dev.capture_begin()
            for j in range(n + 1):
                dev.stamp(j)
                if body is not None and j < n:
                    body()
            g = dev.capture_end()
            per = []
            for _ in range(5):
                dev.graph_launch(g)
                t = dev.stamps_read(0, n + 1)
                per.append((t[n] - t[0]) / n)
            dev.graph_destroy(g)
            res[label] = {"median_us": statistics.median(per), "min_us": min(per), "mean_us": statistics.fmean(per)}
        shapes = [ConvShape(*map(int, s.split())) for s in args.shapes.split(";")]
        wl = Workload(dev, shapes)
        for i, s in enumerate(shapes):
            name = "conv " + " ".join(map(str, s.as_dims()))
            res[name + " [table]"] = timed(dev, lambda: wl.launch(i), args.reps)
        wl.free()
    for k, v in res.items():
        print(f"{k:48s} median {v['median_us']:7.2f} us  min {v['min_us']:7.2f} us")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
