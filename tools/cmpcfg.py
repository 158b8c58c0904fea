#!/usr/bin/env python3
"""Time chosen (config, splits) candidates on chosen ops, the way tools/tune.py does
(amortized over a replayed graph of back-to-back calls), for quick A/B checks.

  python tools/cmpcfg.py --conv "20 96 27 27 256 5 5 1 1 2 2" --cand r128x128x32d2:2 --cand srk128x128x32d2:2
  (a candidate "table" = the committed tuning table's choice)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402
_TUNE_ENV = os.environ.get("BH_TUNE_FILE")
from tools.tune import time_op  # noqa: E402

# the "table" candidate here means the committed table (or the caller's BH_TUNE_FILE); tools.tune
# points BH_TUNE_FILE at nothing only in its own main()
if _TUNE_ENV is None:
    os.environ.pop("BH_TUNE_FILE", None)
else:
    os.environ["BH_TUNE_FILE"] = _TUNE_ENV


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv", action="append", default=[])
    ap.add_argument("--sgemm", action="append", default=[])
    ap.add_argument("--cand", action="append", default=[], help="cfg:splits (or 'table')")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = boda_hip.Device(0)
    shapes = [ops.ConvShape(*map(int, s.split())) for s in a.conv] + \
             [ops.SgemmShape(*map(int, s.split())) for s in a.sgemm]
    for s in shapes:
        kind = 0 if isinstance(s, ops.SgemmShape) else 1
        names = boda_hip.tune_cfg_names(kind)
        wl = runner.Workload(dev, [s])
        rf = runner.roofline_secs(s) * 1e3
        dims = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
        print("== %s %s  roofline %.4f ms" % ("sgemm" if kind == 0 else "conv", " ".join(map(str, dims)), rf))
        for c in a.cand:
            if c == "table":
                dev.tune_set(kind, -1, 0)
            else:
                cn, sp = c.split(":")
                if cn not in names:
                    continue
                dev.tune_set(kind, names.index(cn), int(sp))
            try:
                t = time_op(dev, wl, 0, a.reps)
                print("   %-22s %.4f ms  %5.1f%% of roofline" % (c, t, 100 * rf / t), flush=True)
            except boda_hip.UnsupportedError as e:
                print("   %-22s unsupported: %s" % (c, e))
        dev.tune_set(kind, -1, 0)
        wl.free()
    dev.close()


if __name__ == "__main__":
    main()
