#!/usr/bin/env python3
"""Where a direct-conv config's output differs from the oracle (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import boda_hip  # noqa: E402
from boda_hip import ops  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_conv import run_conv  # noqa: E402

dev = boda_hip.Device(0)
CASES = [(c, d) for c in sys.argv[1].split(",") for d in sys.argv[2].split(";")] if len(sys.argv) > 2 else [
    ("dc11s4x32d2", "1 4 100 224 40 11 11 4 4 1 1")]
for cn, dims in CASES:
    s = ops.ConvShape(*map(int, dims.split()))
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        out = run_conv(dev, s).reshape(s.B, s.OC, s.OH, s.OW)
    except boda_hip.UnsupportedError as e:
        print(cn, dims, "unsup", e)
        continue
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1).reshape(s.B, s.OC, s.OH, s.OW)
    bad = np.abs(out - ref) > 1e-3 * max(1.0, np.abs(ref).max())
    idx = np.argwhere(bad)
    print(cn, dims, "OHxOW", s.OH, s.OW, "bad", len(idx))
    if len(idx):
        print("  oc range", idx[:, 1].min(), idx[:, 1].max(), " oy", sorted(set(idx[:, 2].tolist()))[:20],
              " ox", idx[:, 3].min(), idx[:, 3].max())
dev.tune_set(1, -1, 0)

if os.environ.get("DUMP"):
    s = ops.ConvShape(*map(int, os.environ["DUMP"].split()))
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(os.environ.get("CFG", "dc11s4x32d2")), 0)
    out = run_conv(dev, s).reshape(s.B, s.OC, s.OH * s.OW)
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1).reshape(s.B, s.OC, s.OH * s.OW)
    for oc in range(0, s.OC, 7):
        px = s.OH * s.OW - 1
        got = out[0, oc, px]
        cand = np.argwhere(np.abs(ref[0] - got) < 1e-4 * max(1.0, abs(got)))
        print("oc", oc, "px", px, "got", got, "want", ref[0, oc, px], "got matches ref at", cand[:4].tolist(),
              "neighbours", ref[0, oc, px - 2:px + 1].tolist())
    dev.tune_set(1, -1, 0)
