#!/usr/bin/env python3
"""Timeline of one GEMM/conv call from inside the kernel: with the instrumented build
(make -C boda-1_amd ktrace -> lib/libboda_hip_ktrace.so) thread 0 of every block writes
the device clock at: 0 entry, 1 first K tile in LDS, 2 K loop done, 3 split-K ticket
taken, 4 stores drained. Marks are reported relative to a stamp kernel enqueued just
before the call (and the stamp after it), in microseconds.

  BH_LIB_NAME=libboda_hip_ktrace.so python tools/ktrace.py --conv "1 192 28 28 16 1 1 1 1 0 0" \
      [--cfg 4 --splits 3]
"""
import argparse
import os
import statistics
import sys

os.environ.setdefault("BH_LIB_NAME", "libboda_hip_ktrace.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "boda-1_amd"))

import boda_hip as bh  # noqa: E402
from boda_hip.ops import ConvShape, SgemmShape  # noqa: E402
from boda_hip.runner import Workload  # noqa: E402

BASE = 65535      # pre-call stamp slot; block marks start at BASE + 1 (bh_gemm.hip BH_KTRACE)
NSLOT = 8 * 8192  # marks read back
POST = BASE + 1 + NSLOT


def one(dev, wl, reps):
    rows = []
    for _ in range(reps):
        dev.stamp(BASE)
        wl.launch(0)
        dev.stamp(POST)
        us = dev.stamps_read(BASE, POST - BASE + 1)
        marks = us[1:1 + NSLOT]
        post = us[-1]
        pts = {}
        for k in range(8):
            v = [marks[b * 8 + k] for b in range(NSLOT // 8) if 0 < marks[b * 8 + k] <= post]
            if v:
                pts[k] = v
        # per-block phase durations: prologue (m1-m0), K loop (m2-m1), epilogue (m4-m2)
        dur = {}
        for a, b in ((0, 1), (1, 2), (2, 4), (2, 3), (3, 5), (5, 6), (6, 4)):
            d = [marks[i * 8 + b] - marks[i * 8 + a] for i in range(NSLOT // 8)
                 if 0 < marks[i * 8 + a] <= post and 0 < marks[i * 8 + b] <= post]
            if d:
                dur["%d-%d" % (a, b)] = d
        pts["dur"] = dur
        rows.append((post, pts))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv", action="append", default=[])
    ap.add_argument("--sgemm", action="append", default=[])
    ap.add_argument("--cfg", default="-1", help="config index or name")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    shapes = [ConvShape(*map(int, s.split())) for s in args.conv] + \
             [SgemmShape(*map(int, s.split())) for s in args.sgemm]
    with bh.Device(0) as dev:
        for s in shapes:
            kind = 0 if isinstance(s, SgemmShape) else 1
            ci = int(args.cfg) if args.cfg.lstrip("-").isdigit() else bh.tune_cfg_names(kind).index(args.cfg)
            dev.tune_set(kind, ci, args.splits)
            wl = Workload(dev, [s])
            wl.launch(0)
            dev.sync()
            dims = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
            print("== %s %s  variant %s" % ("sgemm" if kind == 0 else "conv", " ".join(map(str, dims)),
                                          bh.variant_name(kind, dims)))
            for post, pts in one(dev, wl, args.reps)[1:]:
                line = "  post %7.2f |" % post
                for k in range(8):
                    if k in pts:
                        v = pts[k]
                        line += " m%d %6.2f/%6.2f/%6.2f (%d)" % (k, min(v), statistics.median(v), max(v), len(v))
                print(line)
                print("      per-block us (median/max): " + "  ".join(
                    "m%s %.2f/%.2f" % (k, statistics.median(v), max(v)) for k, v in pts["dur"].items()))
            wl.free()
            dev.tune_set(kind, -1, 0)


if __name__ == "__main__":
    main()
