#!/usr/bin/env python3
"""Per-phase shader-clock sums of the Winograd kernel (trace build of bh_wino.hip, -DBH_KTRACE:
[1] wait + barrier, [2] DMA issue, [3] fragment reads + input transform, [4] MFMA issue,
[5] tile epilogues, [6] iterations, [7] whole block), averaged over the grid's blocks.
  BH_LIB_NAME=libboda_hip_wgkt.so python tools/wg_phases.py --conv 20,64,56,56,192,3,3,1,1,1,1 --cfg wg64x64v --splits 5
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv", action="append", default=[])
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--splits", default="1")
    ap.add_argument("--slowest", type=int, default=0, help="also print the N slowest blocks' phases")
    a = ap.parse_args()
    dev = boda_hip.Device(0)
    names = boda_hip.tune_cfg_names(1)
    for c in a.conv:
        s = ops.ConvShape(*map(int, c.split(",")))
        wl = runner.Workload(dev, [s])
        for cn in a.cfg:
            for S in map(int, a.splits.split(",")):
                dev.tune_set(1, names.index(cn), S)
                for _ in range(3):
                    wl.launch(0)
                dev.sync()
                rows = []
                for b in range(2048):
                    v = dev.stamps_read(65536 + 8 * b, 8)
                    cyc = [x * 100.0 for x in v]
                    if cyc[7] <= 0 or cyc[6] <= 0:
                        break
                    rows.append(cyc)
                n = len(rows)
                avg = [sum(r[i] for r in rows) / n for i in range(8)]
                mx = max(r[7] for r in rows)
                print("%s %s S=%d blocks=%d iters/blk %.1f | wait %.0f dma %.0f xf %.0f mfma %.0f epi %.0f "
                      "| total %.0f (max %.0f) cyc; per iter: wait %.0f dma %.0f xf %.0f mfma %.0f" % (
                          c, cn, S, n, avg[6], avg[1], avg[2], 0.0, avg[4], avg[5], avg[7], mx,
                          avg[1] / avg[6], avg[2] / avg[6], 0.0, avg[4] / avg[6]), flush=True)
                if a.slowest:
                    tot = sorted(r[7] for r in rows)
                    print("   total percentiles 10/50/90/99: %.0f %.0f %.0f %.0f" % tuple(
                        tot[min(n - 1, int(q * n))] for q in (0.1, 0.5, 0.9, 0.99)))
                    t0 = min(r[3] for r in rows)  # slot 3: the block's start (absolute)
                    end = [r[3] - t0 + r[7] for r in rows]
                    st = sorted(r[3] - t0 for r in rows)
                    print("   start skew percentiles 50/90/max: %.0f %.0f %.0f; end max %.0f" % (
                        st[n // 2], st[int(0.9 * n)], st[-1], max(end)))
                    for b in sorted(range(n), key=lambda b: -end[b])[:a.slowest]:
                        r = rows[b]
                        print("   block %4d (xcd %d): start %.0f iters %.0f wait %.0f mfma %.0f epi %.0f total %.0f end %.0f" % (
                            b, b % 8, r[3] - t0, r[6], r[1], r[4], r[5], r[7], end[b]))
        dev.tune_set(1, -1, 0)
        wl.free()
    dev.close()


if __name__ == "__main__":
    main()
