#!/usr/bin/env python3
"""Element-wise accuracy of every tuning-table route that is a Winograd variant, on the GPU.

For each conv of the given op lists whose table route (bh_variant_name) is *_wino_*: run it on
mode-5 data through the packed bank, compare with the double-accumulated oracle, print Boda's
element metric max min_sig_mag_rel_diff(1, ref, out) (src/boda_base.cc:140-153) against the
2e-3 Winograd tolerance (src/rtc_prof.cc:314-319), the normalized max and the route. Ops above
--full-max GFLOP compare a --samples-output sample. --all-wx also forces every wx / wg
configuration that runs the op (the tuner's candidates) and prints theirs.

  python tools/wino_gate.py --sets conv,op-sigs,nets > gpurun_out/wino_gate.txt
Tool only (imports the oracle); never on the product path.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)
import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402
from oracle import oracle as orc  # noqa: E402

SETS = {"conv": "tests/golden/ops/conv-ops-1-5-20-nin-alex-gn.txt", "op-sigs": "tests/golden/ops/op_sigs_full.txt",
        "nets": "boda-1_amd/tuning/net-ops-b20.txt", "nets-b5": "boda-1_amd/tuning/net-ops-b5.txt",
        "nets-b1": "boda-1_amd/tuning/net-ops-b1.txt"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="conv,op-sigs,nets,nets-b5,nets-b1")
    ap.add_argument("--full-max", type=float, default=20.0, help="GFLOP above which outputs are sampled")
    ap.add_argument("--samples", type=int, default=1 << 18)
    ap.add_argument("--all-wx", action="store_true")
    ap.add_argument("--force", default="", help="cfg:splits,...: also run these forced routes on every op "
                    "(with --any: on every conv, not only Winograd-eligible ones)")
    ap.add_argument("--any", action="store_true", help="report every op's table route, Winograd or not")
    ap.add_argument("--ops-file", default="", help="an op list file instead of --sets")
    a = ap.parse_args()
    if a.ops_file:
        SETS["file"] = a.ops_file
        a.sets = "file"
    forced = [(f.split(":")[0], int(f.split(":")[1]) if ":" in f else 0) for f in a.force.split(",") if f]
    dev = boda_hip.Device(0)
    names = boda_hip.tune_cfg_names(1)
    seen, worst = set(), 0.0
    for sn in a.sets.split(","):
        o, _ = ops.read_ops(os.path.join(ROOT, SETS[sn]))
        for op in o:
            s = ops.shape_of(op)
            if not isinstance(s, ops.ConvShape) or s in seen:
                continue
            seen.add(s)
            v = dev.variant(1, s.as_dims())
            wx_ok = s.KY == s.KX and s.KY in (3, 5) and s.sy == s.sx == 1 and s.py == s.px <= s.KY // 2
            if "_wino_" not in v and not (a.all_wx and wx_ok) and not a.any:
                continue
            inp, filts, biases = orc.gen_conv(s, 5)
            n = s.B * s.OC * s.OH * s.OW
            if s.flops() <= a.full_max * 1e9:
                idx, ref = None, orc.conv_ref(inp, filts, biases, s, 1)
            else:
                idx = np.random.default_rng(3).choice(n, min(n, a.samples), replace=False).astype(np.uint64)
                ref = orc.conv_ref_at(inp, filts, biases, s, idx, 1)
            wl = runner.Workload(dev, [s])
            routes = [(-1, v, 0)] if ("_wino_" in v or a.any) else []
            if a.all_wx:
                routes += [(ci, cn, 0) for ci, cn in enumerate(names) if cn.startswith(("wx", "wg"))]
            routes += [(names.index(cn), cn, sp) for cn, sp in forced]
            for ci, cn, sp in routes:
                dev.tune_set(1, ci, sp)
                try:
                    wl.launch(0)
                except boda_hip.UnsupportedError:
                    continue
                finally:
                    dev.tune_set(1, -1, 0)
                got = wl.output(0)
                if idx is not None:
                    got = got[idx.astype(np.int64)]
                nm, rl2, hyb = orc.normalized_errors(ref, got)
                if ci < 0 and "_wino_" in cn:
                    worst = max(worst, hyb)
                if sp:
                    cn = "%s:%d" % (cn, sp)
                print("%-44s %-6s elem %.3e %s  norm %.2e  %s%s" % (
                    "x".join(map(str, s.as_dims())), sn, hyb, "FAIL" if hyb > 2e-3 else "ok  ", nm,
                    "table " if ci < 0 else "forced ", cn), flush=True)
            wl.free()
    print("worst table-routed Winograd element error %.3e (tolerance 2e-3)" % worst)
    dev.close()


if __name__ == "__main__":
    main()
