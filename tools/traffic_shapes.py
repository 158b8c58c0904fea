#!/usr/bin/env python3
"""Print the shapes bench.py ran on its dominant kernel (the roofline.kernel variant of a
bench JSON line), one "<kind> <dims>" per line, for the PMC traffic passes. No GPU use."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "boda-1_amd"), ROOT]
import boda_hip  # noqa: E402
from boda_hip import ops  # noqa: E402

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
b = json.loads(line)
kern = b["roofline"]["kernel"]
sets = {"sgemm-ops-full.txt", "conv-ops-1-5-20-nin-alex-gn.txt"}
for fn in b["config"]["workload"].split(" (")[0].split(" + "):
    o, _ = ops.read_ops(os.path.join(ROOT, "tests", "golden", "ops", fn))
    for op in o:
        s = ops.shape_of(op)
        kind = 0 if isinstance(s, ops.SgemmShape) else 1
        d = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
        if boda_hip.variant_name(kind, d) == kern:
            print("sgemm" if kind == 0 else "conv", ",".join(map(str, d)))
