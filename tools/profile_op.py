#!/usr/bin/env python3
"""Run one op repeatedly (for rocprofv3 kernel traces / PMC passes on a single shape).

  python tools/profile_op.py conv 20,64,56,56,192,3,3,1,1,1,1 --cfg 128x128x32 --splits 1 --iters 20
  python tools/profile_op.py sgemm 4096,4096,4096 --iters 10
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["conv", "sgemm"])
    ap.add_argument("dims")
    ap.add_argument("--cfg", default="")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    d = [int(x) for x in a.dims.split(",")]
    kind = 0 if a.kind == "sgemm" else 1
    s = ops.SgemmShape(*d) if kind == 0 else ops.ConvShape(*d)
    dev = boda_hip.Device(0)
    if a.cfg:
        dev.tune_set(kind, boda_hip.tune_cfg_names(kind).index(a.cfg), a.splits)
    wl = runner.Workload(dev, [s])
    wl.launch(0)
    dev.capture_begin()
    dev.stamp(0)
    for _ in range(a.iters):
        wl.launch(0)
    dev.stamp(1)
    g = dev.capture_end()
    per = []
    for _ in range(5):
        dev.graph_launch(g)
        t = dev.stamps_read(0, 2)
        per.append((t[1] - t[0]) / a.iters / 1e3)
    med = sorted(per)[2]
    # eager launches timed on their own kernel dispatches
    ev = []
    for _ in range(5):
        ev.append(dev.time_next_call())
        wl.launch(0)
    dev.sync()
    kt = sorted(dev.elapsed_ms(b, e) for b, e in ev)
    print("kernel-dispatch timed call (median of 5): %.4f ms; back-to-back in a graph (below): per launch" % kt[2])
    print("%s %s cfg=%s splits=%d variant=%s median %.4f ms  %.2f TFLOP/s  roofline %.1f%%" % (
        a.kind, a.dims, a.cfg or "auto", a.splits, boda_hip.variant_name(kind, d), med, s.flops() / med / 1e9,
        100 * runner.roofline_secs(s) * 1e3 / med))
    wl.free()
    dev.close()


if __name__ == "__main__":
    main()
