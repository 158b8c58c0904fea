#!/usr/bin/env python3
"""Time the net executor's HBM-bound layers (bh_fwdops.hip) on the five nets' pooling shapes at
batch 20 and report GB/s of algorithmic bytes (input read once + output written once).

  python tools/layer_bench.py [--json out.json]

Each shape: R calls captured in one hipGraph, replayed warm, timed with events around several
replays (the bench's amortized convention); max pooling without the index output, as
conv_pipe_fwd_t runs it (src/rtc_fwd.cc:263-405).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
import boda_hip  # noqa: E402
from boda_hip import GEN_CONV_IN  # noqa: E402

# (name, B, C, H, W, k, s, p, avg)
POOLS = [("googlenet pool1", 20, 64, 112, 112, 3, 2, 0, 0), ("googlenet pool2", 20, 192, 56, 56, 3, 2, 0, 0),
         ("googlenet inc3 pool", 20, 192, 28, 28, 3, 1, 1, 0), ("googlenet pool3", 20, 480, 28, 28, 3, 2, 0, 0),
         ("googlenet pool4", 20, 832, 14, 14, 3, 2, 0, 0), ("googlenet pool5 avg", 20, 1024, 7, 7, 7, 1, 0, 1),
         ("alexnet pool1", 20, 96, 55, 55, 3, 2, 0, 0), ("alexnet pool2", 20, 256, 27, 27, 3, 2, 0, 0),
         ("alexnet pool5", 20, 256, 13, 13, 3, 2, 0, 0), ("vgg pool1", 20, 64, 224, 224, 2, 2, 0, 0),
         ("vgg pool2", 20, 128, 112, 112, 2, 2, 0, 0), ("resnet pool1", 20, 64, 112, 112, 3, 2, 1, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = boda_hip.Device(0)
    out = []
    for name, B, C, H, W, k, s, p, avg in POOLS:
        OH, OW = boda_hip.pool_out_size(H, k, s, p), boda_hip.pool_out_size(W, k, s, p)
        x, y = dev.alloc_floats(B * C * H * W), dev.alloc_floats(B * C * OH * OW)
        dev.gen_data(GEN_CONV_IN, x, [B, C, H, W], 5)
        dev.capture_begin()
        for _ in range(a.reps):
            dev.pool(x, y, B, C, H, W, k, k, s, s, p, p, avg)
        g = dev.capture_end()
        for _ in range(3):
            dev.graph_launch(g)
        ts = []
        for _ in range(5):
            b = dev.event()
            dev.graph_launch(g)
            e = dev.event()
            dev.sync()
            ts.append(dev.elapsed_ms(b, e) / a.reps)
        dev.graph_destroy(g)
        ms = sorted(ts)[len(ts) // 2]
        nbytes = 4 * (B * C * H * W + B * C * OH * OW)
        r = {"layer": name, "dims": [B, C, H, W, k, s, p, avg], "us": ms * 1e3, "GBps": nbytes / (ms * 1e-3) / 1e9,
             "bytes": nbytes}
        out.append(r)
        print("%-22s %-32s %8.2f us  %7.0f GB/s" % (name, r["dims"], r["us"], r["GBps"]), flush=True)
        x.free()
        y.free()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    dev.close()


if __name__ == "__main__":
    main()
