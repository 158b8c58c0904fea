#!/usr/bin/env python3
"""Graph replay of one libboda_hip call (for the rocprofv3 kernel-trace crash inside
hipGraphLaunch): capture <case> once and replay it 3 times. Cases: gen (gen_data), sgemm, conv
(ring kernel), dm (direct conv), gv (filter streaming), stamp. Diagnostic only.
  rocprofv3 --kernel-trace -d out -o t -- python3 tools/graph_repro.py sgemm"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "boda-1_amd"), ROOT]
import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402

case = sys.argv[1]
dev = boda_hip.Device(0)
if case.startswith("opgraph:"):
    pass
elif case == "gen":
    buf = dev.alloc_floats(1 << 16)
    launch = lambda: dev.gen_data(boda_hip.GEN_SGEMM_A, buf, [256, 256], 5)  # noqa: E731
elif case == "stamp":
    launch = lambda: dev.stamp(0)  # noqa: E731
elif case.startswith("set:"):  # set:<ops file>:<first>:<count> -- one graph of several ops
    _, fn, a, n = case.split(":")
    o, _ = ops.read_ops(os.path.join(ROOT, "tests", "golden", "ops", fn))
    wl = runner.Workload(dev, [ops.shape_of(x) for x in o][int(a):int(a) + int(n)], mode=5)
    launch = wl.step  # noqa: E731
elif case.startswith("conv:"):
    wl = runner.Workload(dev, [ops.ConvShape(*map(int, case[5:].split(",")))])
    launch = lambda: wl.launch(0)  # noqa: E731
else:
    s = {"sgemm": ops.SgemmShape(1024, 1024, 1024), "conv": ops.ConvShape(5, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2),
         "dm": ops.ConvShape(20, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1),
         "gv": ops.ConvShape(1, 512, 14, 14, 128, 1, 1, 1, 1, 0, 0)}[case]
    wl = runner.Workload(dev, [s])
    launch = lambda: wl.launch(0)  # noqa: E731
if case.startswith("opgraph:"):  # opgraph:<ops file>:<count>: bench.py's per-op graph timing (runner.op_graph_time)
    _, fn, n = case.split(":")
    o, _ = ops.read_ops(os.path.join(ROOT, "tests", "golden", "ops", fn))
    wl = runner.Workload(dev, [ops.shape_of(x) for x in o][:int(n)], mode=5)
    wl.step()
    dev.sync()
    for i in range(int(n)):
        t = wl.op_graph_time(i, 100)
        dev.events_reset()
        print("op", i, "%.2f us" % (t * 1e6), flush=True)
    dev.close()
    sys.exit(0)
ngraphs = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # graphs captured, then replayed back to back
launch()
dev.sync()
gs = []
for _ in range(ngraphs):
    dev.capture_begin()
    launch()
    gs.append(dev.capture_end())
print(case, "captured", ngraphs, flush=True)
for r in range(3):
    for g in gs:
        dev.graph_launch(g)
    dev.sync()
    print(case, "replay", r, "ok", flush=True)
for g in gs:
    dev.graph_destroy(g)
dev.close()
