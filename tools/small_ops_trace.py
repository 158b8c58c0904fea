#!/usr/bin/env python3
"""Split each small conv op's per-call time into kernel duration and dispatch gap.

Run under a kernel trace (one process; the ops are replayed as the bench's per-op timing does it:
a hipGraph of N back-to-back calls behind a spin kernel):

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sot -o sot -- \\
      python3 tools/small_ops_trace.py --batch 1 --reps 40 --out gpurun_out/sot_ops.json
  python3 tools/small_ops_trace.py --parse gpurun_out/sot --ops gpurun_out/sot_ops.json \\
      --json profiles/r04/small_ops_trace.json

The first form runs the ops and writes, per op, its position in the launch order; --parse reads the
kernel trace, groups each op's replayed main-kernel dispatches (the op's graph is the only work
between two spin kernels), and reports per op: the amortized per-call time (first start to last end
of the replay / N), the kernel duration (mean end - start), and the gap (per-call time - duration).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

SETS_DIR = os.path.join(ROOT, "tests", "golden", "ops")


def run(a):
    import boda_hip  # noqa: F401
    from boda_hip import ops, runner
    o, _ = ops.read_ops(os.path.join(SETS_DIR, "conv-ops-1-5-20-nin-alex-gn.txt"))
    shapes = [ops.shape_of(x) for x in o]
    shapes = [s for s in shapes if isinstance(s, ops.ConvShape) and s.B in a.batch]
    dev = boda_hip.Device(0)
    rec = []
    for s in shapes:
        wl = runner.Workload(dev, [s])
        wl.launch(0)  # eager first call: grows the split-K workspace outside the capture
        dev.sync()
        # as runner.op_graph_time, with a spin kernel after the timed replay too, so that the trace
        # reads: warm replay | spin | timed replay | spin (segment 2 i + 1 is op i's timed replay)
        dev.capture_begin()
        try:
            for _ in range(a.reps):
                wl.launch(0)
        finally:
            g = dev.capture_end()
        dev.graph_launch(g)
        dev.spin(50)
        b = dev.event()
        dev.graph_launch(g)
        e = dev.event()
        dev.spin(10)
        dev.sync()
        rec.append({"dims": list(s.as_dims()), "graph_us": dev.elapsed_ms(b, e) * 1e3 / a.reps, "reps": a.reps})
        dev.events_reset()
        dev.graph_destroy(g)
        wl.free()
    dev.close()
    json.dump(rec, open(a.out, "w"), indent=0)


def parse(a):
    rec = json.load(open(a.ops))
    rows = []
    for f in glob.glob(os.path.join(a.parse, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # segments between spin kernels; each op contributes: [warm replay] spin [timed replay]
    segs, cur = [], []
    for r in rows:
        if "spin" in r["Kernel_Name"]:
            segs.append(cur)
            cur = []
        else:
            cur.append(r)
    segs.append(cur)
    # segments: warm(0) | timed(0) | warm(1) | timed(1) | ... (spins separate them)
    out = []
    for i, op in enumerate(rec):
        n = op["reps"]
        if 2 * i + 1 >= len(segs):
            break
        sg = segs[2 * i + 1]
        if not sg or len(sg) % n:
            continue
        per = len(sg) // n  # kernels per call (combine kernels included)
        t0, t1 = int(sg[0]["Start_Timestamp"]), int(sg[-1]["End_Timestamp"])
        call_ns = (t1 - t0) / n
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sg]
        kern_ns = sum(dur) / n
        out.append({"dims": op["dims"], "kernels_per_call": per, "kernel": sg[0]["Kernel_Name"][:80],
                    "call_us": round(call_ns / 1e3, 3), "kernel_us": round(kern_ns / 1e3, 3),
                    "gap_us": round((call_ns - kern_ns) / 1e3, 3), "graph_us": round(op["graph_us"], 3)})
    summ = {}
    if out:
        summ = {"ops": len(out),
                "median_call_us": statistics.median(x["call_us"] for x in out),
                "median_kernel_us": statistics.median(x["kernel_us"] for x in out),
                "median_gap_us": statistics.median(x["gap_us"] for x in out),
                "sum_call_us": round(sum(x["call_us"] for x in out), 2),
                "sum_kernel_us": round(sum(x["kernel_us"] for x in out), 2)}
    res = {"summary": summ, "ops": out,
           "method": "rocprofv3 --kernel-trace of tools/small_ops_trace.py: each op replayed as a hipGraph of "
                     "reps back-to-back calls behind a spin kernel (the bench's per-op timing); call = replay "
                     "span / reps, kernel = mean dispatch duration x kernels per call, gap = call - kernel"}
    json.dump(res, open(a.json, "w"), indent=1)
    print(json.dumps(summ, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="1", help="comma list of batch sizes")
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--out", default="gpurun_out/sot_ops.json")
    ap.add_argument("--parse", default="", help="trace directory (second form)")
    ap.add_argument("--ops", default="gpurun_out/sot_ops.json")
    ap.add_argument("--json", default="profiles/r04/small_ops_trace.json")
    a = ap.parse_args()
    a.batch = [int(x) for x in str(a.batch).split(",")]
    if a.parse:
        parse(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
