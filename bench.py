#!/usr/bin/env python3
"""bench.py -- Boda per-op conv/SGEMM hot path on MI355X.

Metric (BASELINE.json): per-op GFLOPS and % fp32 roofline on sgemm-ops-full +
conv-ops (AlexNet/NiN/GoogLeNet). A "step" is one pass over the workload's op
list, one main-kernel launch per op, inputs resident in HBM (generated on the
device with the reference's gen_data mode 5 before the timed region).

  value       = sum of algorithmic flops of every op launched on every rank in
                the timed steps / max-over-ranks wall time    [GFLOP/s]
  per_set     = per op-list aggregate in the reference's own convention:
                sum flops / sum per-op GPU seconds (src/rtc_prof.cc:104-124),
                plus sum(roofline time) / sum(kernel time)
  launch      = each timed step is a captured hipGraph (no host launch latency
                between ops; --eager for op-by-op launches from Python)
  roofline    = the dominant kernel (most time): algorithmic flops per launch / its
                average launch duration, measured with HIP events on the kernel's
                stream around a replayed graph of back-to-back calls, vs fp32 peak
  cpu_baseline= the oracle's fp32 OpenMP CPU implementation (kind "port") on a
                bounded sample, rank 0 at N=1 only

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
ops are independent so there is no data-path collective; every
rank runs one full copy of the op list on its own GPU (weak scaling), a gloo
barrier brackets the timed region and the max wall time over ranks is used.
--strong instead shards ONE op list over the ranks (greedy LPT on roofline time).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402
from boda_hip.shard import Dist, lpt_partition  # noqa: E402

OPS_DIR = os.path.join(ROOT, "tests", "golden", "ops")
SETS = {
    "sgemm-full": "sgemm-ops-full.txt",
    "sgemm-small": "sgemm-ops-small.txt",
    "sgemm-tiny": "sgemm-ops-tiny.txt",
    "conv": "conv-ops-1-5-20-nin-alex-gn.txt",
    "op-sigs": "op_sigs_full.txt",
}
DEFAULT_SETS = ["sgemm-full", "conv"]


def load_sets(names):
    shapes, tags = [], []
    for n in names:
        o, _ = ops.read_ops(os.path.join(OPS_DIR, SETS[n]))
        for op in o:
            shapes.append(ops.shape_of(op))
            tags.append(n)
    return shapes, tags


def cpu_baseline(budget_s):
    """Time the oracle's fp32 OpenMP CPU path on a bounded sample of the same workload."""
    from oracle import oracle as orc
    conv, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["conv"]))
    sg, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["sgemm-small"]))
    sgf, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["sgemm-full"]))
    # every conv op, then the SGEMMs smallest first until the time budget is spent
    sample = [ops.shape_of(o) for o in conv]
    sample += sorted({ops.shape_of(o) for o in sg + sgf}, key=lambda s: s.flops())
    flops = secs = 0.0
    done = 0
    for s in sample:
        if isinstance(s, ops.SgemmShape):
            a, b = orc.gen_sgemm(s.M, s.N, s.K, 5)
            t0 = time.perf_counter()
            orc.sgemm_ref(a, b, s.M, s.N, s.K, fast=True)
        else:
            i, f, b = orc.gen_conv(s, 5)
            t0 = time.perf_counter()
            orc.conv_ref(i, f, b, s, 1, fast=True)
        secs += time.perf_counter() - t0
        flops += s.flops()
        done += 1
        if secs > budget_s:
            break
    return {"value": round(flops / secs / 1e9, 3), "unit": "GFLOP/s", "cores": orc.num_threads(), "kind": "port",
            "sample": "%d of %d ops: all 204 conv-ops-1-5-20 + sgemm-ops-small/full smallest first until the "
                      "%.0f s budget, fp32, %.1f GFLOP in %.1f s" % (done, len(sample), budget_s, flops / 1e9, secs)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", default=",".join(DEFAULT_SETS))
    ap.add_argument("--strong", action="store_true", help="shard one op list over the ranks (LPT)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--per-op", default="", help="write per-op event times (JSON) to this path")
    ap.add_argument("--eager", action="store_true", help="launch op by op from Python instead of hipGraph replay")
    ap.add_argument("--op-timing", choices=["graph", "events"], default="graph",
                    help="per-op time: amortized over a replayed graph of back-to-back calls (default), or HIP "
                         "events bound to each call's own dispatches")
    args = ap.parse_args()

    dd = Dist()
    if dd.world != args.gpus:
        if args.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d ranks" % (args.gpus, args.gpus))
    set_names = [s for s in args.sets.split(",") if s]
    shapes, tags = load_sets(set_names)
    if args.strong and dd.world > 1:
        mine = lpt_partition([runner.roofline_secs(s) for s in shapes], dd.world)[dd.rank]
    else:
        mine = list(range(len(shapes)))
    my_shapes = [shapes[i] for i in mine]
    my_tags = [tags[i] for i in mine]

    # one GPU per rank; ranks beyond the node's GPU count share (rehearsal on a 1-GPU box)
    dev = boda_hip.Device(dd.local_rank % max(1, boda_hip.device_count()))
    wl = runner.Workload(dev, my_shapes, mode=5, tags=my_tags)
    for _ in range(args.warmup):
        wl.step()
    dev.sync()

    # Timed region: K steps, each a captured hipGraph of the whole op sweep, replayed
    # back to back (--eager: launched op by op from Python instead).
    nop = len(my_shapes)
    graphs = [] if args.eager else [wl.capture_step() for _ in range(args.steps)]
    dd.barrier()
    dev.sync()
    t0 = time.perf_counter()
    if args.eager:
        for _ in range(args.steps):
            wl.step()
    else:
        for g in graphs:
            dev.graph_launch(g)
    dev.sync()
    t1 = time.perf_counter()
    dd.barrier()
    elapsed = dd.max(t1 - t0)

    # Per-op GPU time (the reference's per-op convention, src/rtc_prof.cc:104-124): K more
    # steps, each op timed by HIP events recorded on its own first/last kernel dispatch.
    # With --op-timing graph (default) those are only the estimate that sizes a replayed
    # graph of back-to-back calls per op, whose amortized per-call time is what we report.
    events = []
    for _ in range(args.steps):
        wl.step_kernel_timed(events)
    dev.sync()
    ktime = [0.0] * nop
    for i, b, e in events:
        ktime[i] += dev.elapsed_ms(b, e) / 1e3
    dev.events_reset()
    ktime = [t / args.steps for t in ktime]
    ev_time = list(ktime)
    if args.op_timing == "graph":
        for i in range(nop):
            reps = max(3, min(100, int(round(2e-3 / max(ktime[i], 1e-6)))))
            ktime[i] = wl.op_graph_time(i, reps)
            dev.events_reset()

    my_flops = sum(s.flops() for s in my_shapes)
    total_flops = dd.sum(my_flops) * args.steps
    value = total_flops / elapsed / 1e9

    per_set = {}
    for n in set_names:
        idx = [i for i, t in enumerate(my_tags) if t == n]
        if not idx:
            continue
        f = sum(my_shapes[i].flops() for i in idx)
        t = sum(ktime[i] for i in idx)
        rt = sum(runner.roofline_secs(my_shapes[i]) for i in idx)
        per_set[n] = {"ops": len(idx), "gflop": round(f / 1e9, 3), "sum_kernel_ms": round(t * 1e3, 4),
                      "gflops": round(f / t / 1e9, 2), "roofline_frac": round(rt / t, 4),
                      "roofline_ms": round(rt * 1e3, 4)}

    # dominant kernel: the variant with the most event time
    by_var = {}
    for i, s in enumerate(my_shapes):
        kind = 0 if isinstance(s, ops.SgemmShape) else 1
        dims = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
        v = boda_hip.variant_name(kind, dims)
        d = by_var.setdefault(v, {"t": 0.0, "flops": 0.0, "bytes": 0.0, "n": 0})
        d["t"] += ktime[i]
        d["flops"] += s.flops()
        d["bytes"] += s.bytes()
        d["n"] += 1
    dom = max(by_var, key=lambda v: by_var[v]["t"])
    dv = by_var[dom]
    achieved = dv["flops"] / dv["t"] / 1e12
    roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": runner.PEAK_FP32_FLOPS / 1e12,
            "unit": "TFLOP/s", "frac": round(achieved * 1e12 / runner.PEAK_FP32_FLOPS, 4), "traffic": None,
            "launches_per_step": dv["n"], "avg_launch_ms": round(dv["t"] / dv["n"] * 1e3, 4),
            "avg_flops_per_launch": dv["flops"] / dv["n"]}
    tp = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tp):
        try:
            tj = json.load(open(tp))
            if tj.get("kernel") == dom:
                roof["traffic"] = tj.get("bytes_per_launch")
                roof["traffic_source"] = tj.get("source")
        except (OSError, ValueError):
            pass

    cpu = None
    if dd.rank == 0 and dd.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_budget)

    if args.per_op and dd.rank == 0:
        with open(args.per_op, "w") as f:
            json.dump([{"tag": my_tags[i], "dims": (my_shapes[i].as_dims() if isinstance(my_shapes[i], ops.ConvShape)
                                                   else [my_shapes[i].M, my_shapes[i].N, my_shapes[i].K]),
                        "kernel_ms": ktime[i] * 1e3, "event_ms": ev_time[i] * 1e3, "gflops": my_shapes[i].flops() / ktime[i] / 1e9,
                        "roofline_frac": runner.roofline_secs(my_shapes[i]) / ktime[i],
                        "bound": runner.bound_of(my_shapes[i])} for i in range(len(my_shapes))], f, indent=0)

    if dd.rank == 0:
        line = {
            "metric": "per-op GFLOPS and % fp32 roofline on sgemm-ops-full + conv-ops (AlexNet/NiN/GoogLeNet)",
            "value": round(value, 2), "unit": "GFLOP/s", "n_gpus": dd.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if (args.strong and dd.world > 1) else "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (reference gen_data mode 5, generated on device)",
            "config": {"workload": " + ".join(SETS[n] for n in set_names) + " (one main-kernel launch per op per step)",
                       "launch": "eager" if args.eager else "hipGraph replay of each step",
                       "op_timing": ("per-op amortized time over a replayed hipGraph of back-to-back calls, "
                                     "HIP events around the replay (after the timed region)"
                                     if args.op_timing == "graph" else
                                     "HIP events on each op's first/last kernel dispatch (hipExtLaunchKernel), "
                                     "K extra eager steps after the timed region"),
                       "ops_per_gpu": len(my_shapes), "gflop_per_step_per_gpu": round(my_flops / 1e9, 3),
                       "parallelism": ("op-shard" if args.strong else "op-replica") + "%d" % dd.world,
                       "plat": dev.plat_tag()},
            "per_set": per_set,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    for g in graphs:
        dev.graph_destroy(g)
    wl.free()
    dev.close()
    dd.close()


if __name__ == "__main__":
    main()
