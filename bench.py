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
  vendor      = per_set.*.vendor_ms: rocBLAS sgemm / MIOpen conv+bias+ReLU on the same units and
                in the same amortized convention (libboda_hip_vendor.so), a same-node yardstick
                only (--vendor off skips it)
  cpu_baseline= the oracle's fp32 OpenMP CPU implementation (kind "port") on a
                bounded sample, rank 0 at N=1 only

Workload: sgemm-ops-full + conv-ops-1-5-20 (the metric's two lists, BASELINE configs C2/C3)
+ op_sigs_full (C5) -- the same fixed list at every N, so per-N values compare directly.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): ops are
independent (src/rtc_prof.cc:232-360), so the list is SHARDED over the ranks
with no data-path collective: greedy LPT on roofline time (boda_hip/shard.py, the algorithm of
boda_hip_ops_prof --shard=k/n), SGEMMs bigger than half a rank's share first cut into column
panels (independent M x n_j x K sub-ops). Each rank runs its units on its own GPU; a gloo
barrier brackets the timed region and the max wall time over ranks is used ("scaling":
"strong": the total work is fixed). The line carries the predicted LPT imbalance (max rank
roofline load / mean) and the measured one (max rank wall time / mean). More ranks than GPUs
is refused unless --rehearsal (then "shared_device": true).
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
from boda_hip.shard import Dist, imbalance, lpt_partition, plan_units  # noqa: E402

OPS_DIR = os.path.join(ROOT, "tests", "golden", "ops")
SETS = {
    "sgemm-full": "sgemm-ops-full.txt",
    "sgemm-small": "sgemm-ops-small.txt",
    "sgemm-tiny": "sgemm-ops-tiny.txt",
    "conv": "conv-ops-1-5-20-nin-alex-gn.txt",
    "op-sigs": "op_sigs_full.txt",
}
DEFAULT_SETS = ["sgemm-full", "conv", "op-sigs"]


def load_sets(names):
    shapes, tags = [], []
    for n in names:
        o, _ = ops.read_ops(os.path.join(OPS_DIR, SETS[n]))
        for op in o:
            shapes.append(ops.shape_of(op))
            tags.append(n)
    return shapes, tags


def shard_units(shapes, tags, world, rank):
    """This rank's units of the sharded sweep: (all units, my units, predicted LPT imbalance)."""
    costs = [runner.roofline_secs(s) for s in shapes]
    units = plan_units(shapes, costs, world)
    parts = lpt_partition([u[2] for u in units], world)
    pred = imbalance([sum(units[i][2] for i in p) for p in parts])
    return units, [units[i] for i in parts[rank]], pred


def build_hash():
    """sha256 over the kernel sources and the tuning table: what decides which kernel runs each unit
    and how fast (a committed rocprof figure is reported only for the build it was measured on)."""
    import hashlib
    h = hashlib.sha256()
    src = os.path.join(ROOT, "boda-1_amd", "csrc")
    for fn in sorted(os.listdir(src)):
        if fn.endswith((".hip", ".h")):
            h.update(fn.encode())
            h.update(open(os.path.join(src, fn), "rb").read())
    h.update(open(os.path.join(ROOT, "boda-1_amd", "tuning", "gfx950.tune"), "rb").read())
    return h.hexdigest()[:16]


def cpu_info():
    """Host facts for the CPU baseline line: logical CPUs, the CPUs this process may run on, the
    CPU model string."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for l in f:
                if l.startswith("model name"):
                    model = l.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"nproc": os.cpu_count(), "affinity": aff, "cpu_model": model}


def executed_flops(s, variant):
    """Flops an op's kernel actually issues: a Winograd route multiplies its transformed input values by
    the transformed filter values position by position, per output tile and (input, output) channel
    pair (outputs computed up to a whole number of tiles), the other routes the direct-form 2*M*N*K
    of src/latex-util.H:116-120 (SGEMM: 2*M*N*K)."""
    if "_wino_" in variant:
        # wx43: F(4x4, 3x3), 36 products per 4x4 tile; wx25: F(2x2, 5x5), 36 per 2x2 tile; wg* / wx23:
        # F(2x2, 3x3), 16 per 2x2 tile
        mo, pos = (4, 36) if "_wino_wx43" in variant else ((2, 36) if "_wino_wx25" in variant else (2, 16))
        tiles = s.B * (-(-s.OH // mo)) * (-(-s.OW // mo))
        return 2.0 * pos * s.OC * s.IC * tiles
    return s.flops()


def cpu_baseline(budget_s):
    """Time the oracle's fp32 OpenMP CPU path on a bounded sample of the same workload: every op
    of conv-ops-1-5-20 and op_sigs_full, then the SGEMMs of sgemm-ops-small/full smallest first
    until the time budget is spent."""
    from oracle import oracle as orc
    conv, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["conv"]))
    sigs, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["op-sigs"]))
    sg, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["sgemm-small"]))
    sgf, _ = ops.read_ops(os.path.join(OPS_DIR, SETS["sgemm-full"]))
    sample = [ops.shape_of(o) for o in conv] + [ops.shape_of(o) for o in sigs]
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
    info = cpu_info()
    nt = orc.num_threads()
    why = ("OMP_NUM_THREADS" if os.environ.get("OMP_NUM_THREADS") else "the OpenMP default")
    line = {"value": round(flops / secs / 1e9, 3), "unit": "GFLOP/s", "cores": nt, "kind": "port",
            "sample": "%d of %d ops: all 204 conv-ops-1-5-20 + 178 op_sigs_full ops, then sgemm-ops-small/full "
                      "smallest first until the %.0f s budget; fp32 OpenMP, %d threads (%s; the GPU box grants "
                      "each one-GPU lease a share of 16 CPUs although its affinity mask lists %s, so the "
                      "baseline runs on that share, not on every listed CPU), %.1f GFLOP in %.1f s"
                      % (done, len(sample), budget_s, nt, why, info["affinity"], flops / 1e9, secs)}
    line.update(info)
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", default=",".join(DEFAULT_SETS))
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than GPUs (ranks share devices; the line says shared_device)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--per-op", default="", help="write per-unit times (JSON, all ranks) to this path")
    ap.add_argument("--eager", action="store_true", help="launch op by op from Python instead of hipGraph replay")
    ap.add_argument("--op-timing", choices=["graph", "events"], default="graph",
                    help="per-op time: amortized over a replayed graph of back-to-back calls (default), or HIP "
                         "events bound to each call's own dispatches")
    ap.add_argument("--vendor", choices=["on", "off"], default="on",
                    help="also time rocBLAS sgemm / MIOpen conv(+bias+ReLU) per unit (libboda_hip_vendor.so): "
                         "per_set.*.vendor_ms, context only")
    args = ap.parse_args()

    dd = Dist()
    if dd.world != args.gpus:
        sys.exit("--gpus %d needs torch.distributed.run with %d ranks (got world size %d)" % (args.gpus, args.gpus,
                                                                                        dd.world))
    ndev = boda_hip.device_count()
    shared = dd.max(1.0 if dd.local_rank >= ndev else 0.0) > 0  # some rank has no GPU of its own
    if shared and not args.rehearsal:
        sys.exit("rank %d: local rank %d but only %d GPU(s); pass --rehearsal to let ranks share a device"
                 % (dd.rank, dd.local_rank, ndev))
    set_names = [s for s in args.sets.split(",") if s]
    shapes, tags = load_sets(set_names)
    units, mine, pred_imb = shard_units(shapes, tags, dd.world, dd.rank)
    my_shapes = [u[1] for u in mine]
    my_tags = [tags[u[0]] for u in mine]

    dev = boda_hip.Device(dd.local_rank % max(1, ndev))
    wl = runner.Workload(dev, my_shapes, mode=5, tags=my_tags)
    for _ in range(args.warmup):
        wl.step()
    dev.sync()

    # Timed region: K steps, each a captured hipGraph of this rank's sweep, replayed back to
    # back (--eager: launched op by op from Python instead).
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
    rank_times = dd.gather_obj(t1 - t0)

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

    # Same-node comparator (context, never the target): the vendor libraries on the same units, in
    # the same amortized back-to-back convention (src/culibs-wrap.cc:94-242 is the reference's seam).
    vtime = [None] * nop
    vinfo = [None] * nop
    vendor_note = None
    if args.vendor == "on":
        from boda_hip import vendor
        if not os.path.exists(vendor.LIB_PATH):  # comparator not built: the line says so
            vendor_note = "libboda_hip_vendor.so not built: vendor_ms null"
        else:
            vd = vendor.Vendor(dd.local_rank % max(1, ndev))
            for i in range(nop):
                reps = max(3, min(50, int(round(2e-3 / max(ktime[i], 1e-6)))))
                vinfo[i] = vd.time(my_shapes[i], reps)
                vtime[i] = vinfo[i]["ms"] / 1e3
            vd.close()

    my_flops = sum(s.flops() for s in my_shapes)
    total_flops = dd.sum(my_flops) * args.steps
    value = total_flops / elapsed / 1e9

    # every rank's per-unit records, gathered on rank 0 (per-set sums and the dominant kernel are
    # over the whole job)
    recs = []
    for i, s in enumerate(my_shapes):
        kind = 0 if isinstance(s, ops.SgemmShape) else 1
        dims = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
        recs.append({"tag": my_tags[i], "op": mine[i][0], "dims": dims, "variant": boda_hip.variant_name(kind, dims),
                     "flops": s.flops(), "bytes": s.bytes(), "kernel_s": ktime[i], "event_s": ev_time[i],
                     "roof_s": runner.roofline_secs(s), "bound": runner.bound_of(s), "rank": dd.rank,
                     "vendor_s": vtime[i], "vendor": vinfo[i]})
        fx = executed_flops(s, recs[-1]["variant"])
        recs[-1].update({"flops_executed": fx,
                         "roof_exec_s": max(fx / runner.PEAK_FP32_FLOPS, s.bytes() / runner.PEAK_HBM_BPS)})
    recs = [r for part in dd.gather_obj(recs) for r in part]

    per_set = {}
    for n in set_names:
        rs = [r for r in recs if r["tag"] == n]
        if not rs:
            continue
        f = sum(r["flops"] for r in rs)
        t = sum(r["kernel_s"] for r in rs)
        rt = sum(r["roof_s"] for r in rs)
        te = sum(r["event_s"] for r in rs)
        per_set[n] = {"ops": len({r["op"] for r in rs}), "gflop": round(f / 1e9, 3), "sum_kernel_ms": round(t * 1e3, 4),
                      "gflops": round(f / t / 1e9, 2), "roofline_frac": round(rt / t, 4),
                      "roofline_ms": round(rt * 1e3, 4),
                      # the reference's own per-call convention (event pair around each call)
                      "sum_event_ms": round(te * 1e3, 4), "roofline_frac_events": round(rt / te, 4)}
        # ops on the Winograd route (fewer MFMA flops than the direct flop model the roofline
        # counts): their count and time
        wr = [r for r in rs if "_wino_" in r.get("variant", "")]
        if wr:
            per_set[n].update({"wino_ops": len(wr), "wino_kernel_ms": round(sum(r["kernel_s"] for r in wr) * 1e3, 4)})
        # the same fraction with every op's roofline at the flops its kernel issues (Winograd ops at
        # their transformed-domain products; the headline keeps the reference's direct-form model)
        rx = sum(r["roof_exec_s"] for r in rs)
        per_set[n].update({"roofline_ms_executed": round(rx * 1e3, 4), "roofline_frac_executed": round(rx / t, 4)})
        if all(r["vendor_s"] is not None for r in rs):
            tv = sum(r["vendor_s"] for r in rs)
            per_set[n].update({"vendor_ms": round(tv * 1e3, 4), "vendor_roofline_frac": round(rt / tv, 4),
                               "vendor_over_ours": round(tv / t, 3),
                               "ops_faster_than_vendor": sum(r["kernel_s"] <= r["vendor_s"] for r in rs)})

    # dominant kernel: the variant with the most time over the whole job
    by_var = {}
    for r in recs:
        d = by_var.setdefault(r["variant"], {"t": 0.0, "flops": 0.0, "fx": 0.0, "bytes": 0.0, "n": 0})
        d["t"] += r["kernel_s"]
        d["flops"] += r["flops"]
        d["fx"] += r.get("flops_executed", r["flops"])
        d["bytes"] += r["bytes"]
        d["n"] += 1
    dom = max(by_var, key=lambda v: by_var[v]["t"])
    dv = by_var[dom]
    achieved = dv["flops"] / dv["t"] / 1e12
    roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": runner.PEAK_FP32_FLOPS / 1e12,
            "unit": "TFLOP/s", "frac": round(achieved * 1e12 / runner.PEAK_FP32_FLOPS, 4), "traffic": None,
            "launches_per_step": dv["n"], "avg_launch_ms": round(dv["t"] / dv["n"] * 1e3, 4),
            "avg_flops_per_launch": dv["flops"] / dv["n"]}
    if dv["fx"] != dv["flops"]:  # Winograd: the MFMA flops the kernel actually executes (section 5 of DESIGN.md)
        roof["achieved_executed"] = round(dv["fx"] / dv["t"] / 1e12, 3)
        roof["frac_executed"] = round(dv["fx"] / dv["t"] / runner.PEAK_FP32_FLOPS, 4)
    tp = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tp):
        try:
            tj = json.load(open(tp))
            if tj.get("kernel") == dom:
                roof["traffic"] = tj.get("bytes_per_launch")
                roof["traffic_source"] = tj.get("source")
        except (OSError, ValueError):
            pass
    # the same kernel's average launch duration from the committed rocprofv3 --kernel-trace --stats
    # summary of the graph-replayed step (tools/rocprof_dominant.py): the profile-derived fraction
    # beside the bench's amortized one
    rp = os.path.join(ROOT, "profiles", "rocprof_dominant.json")
    if os.path.exists(rp):
        try:
            rj = json.load(open(rp))
            dom_units = sorted(r["dims"] for r in recs if r["variant"] == dom)
            same = rj.get("units") == dom_units and rj.get("build_hash") == build_hash()
            if rj.get("kernel") == dom and rj.get("avg_ns") and not same:
                roof["frac_rocprof_stale"] = ("profiles/rocprof_dominant.json was measured on another build or "
                                              "other launches of this kernel: not reported")
            if rj.get("kernel") == dom and rj.get("avg_ns") and same:
                a_rp = roof["avg_flops_per_launch"] / (rj["avg_ns"] * 1e-9)
                roof["avg_launch_ms_rocprof"] = round(rj["avg_ns"] * 1e-6, 4)
                roof["frac_rocprof"] = round(a_rp / runner.PEAK_FP32_FLOPS, 4)
                roof["rocprof_source"] = rj.get("source")
        except (OSError, ValueError, KeyError):
            pass

    cpu = None
    if dd.rank == 0 and dd.world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_budget)

    if args.per_op and dd.rank == 0:
        with open(args.per_op, "w") as f:
            json.dump([dict(r, kernel_ms=r["kernel_s"] * 1e3, event_ms=r["event_s"] * 1e3,
                            vendor_ms=None if r["vendor_s"] is None else r["vendor_s"] * 1e3,
                            gflops=r["flops"] / r["kernel_s"] / 1e9, roofline_frac=r["roof_s"] / r["kernel_s"],
                            roofline_frac_executed=r["roof_exec_s"] / r["kernel_s"])
                       for r in recs], f, indent=0)

    if dd.rank == 0:
        n_split = len({u[0] for u in units if u[1] != shapes[u[0]]})
        line = {
            "metric": "per-op GFLOPS and % fp32 roofline on sgemm-ops-full + conv-ops (AlexNet/NiN/GoogLeNet)",
            "metric_note": "value aggregates the three lists of config.workload (the metric's two plus op_sigs_full, "
                           "BASELINE config C5); per_set holds each list's own figures",
            "value": round(value, 2), "unit": "GFLOP/s", "n_gpus": dd.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (reference gen_data mode 5, generated on device)",
            "config": {"workload": " + ".join(SETS[n] for n in set_names) + " (one main-kernel launch per op per step)",
                       "launch": "eager" if args.eager else "hipGraph replay of each step",
                       "op_timing": ("per-op amortized time over a replayed hipGraph of back-to-back calls, "
                                     "HIP events around the replay (after the timed region)"
                                     if args.op_timing == "graph" else
                                     "HIP events on each op's first/last kernel dispatch (hipExtLaunchKernel), "
                                     "K extra eager steps after the timed region"),
                       "ops": len(shapes), "units": len(units), "ops_cut_into_panels": n_split,
                       "panel_operands": "each column panel (M x n_j x K) owns contiguous a (K x M), b (K x n_j) "
                                         "and c (M x n_j); no strided slice of a shared b",
                       "gflop_per_step": round(sum(s.flops() for s in shapes) / 1e9, 3),
                       "parallelism": "op-shard%d (LPT, no collective)" % dd.world,
                       "lpt_imbalance_predicted": round(pred_imb, 4),
                       "lpt_imbalance_measured": round(imbalance(rank_times), 4),
                       "shared_device": shared,
                       "plat": dev.plat_tag(),
                       "vendor": ("rocblas_sgemm / MIOpen Find-chosen conv fwd + miopenOpTensor bias + "
                                  "miopenActivationForward ReLU, same units, amortized back-to-back calls, "
                                  "context only" if args.vendor == "on" and not vendor_note else vendor_note)},
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
