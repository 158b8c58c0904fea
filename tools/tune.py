#!/usr/bin/env python3
"""Sweep tile configurations x K-splits per op on the GPU and write the tuning table.

The backend's counterpart of Boda's op_tune sweeps + wisdom (src/rtc_prof.cc
ops-prof over several --op-tunes; src/op-tuner.cc): for every op of the given
op lists, time each instantiated tile configuration with each split count
(amortized over a replayed graph of back-to-back calls, as bench.py reports
per-op time; --timing flush: median over --reps calls, each after a cache flush,
timed by events on the call's own kernel dispatches), keep the fastest and
write boda-1_amd/tuning/gfx950.tune lines "<op> <dims> cfg=<name> splits=<n>".
Results of every candidate go to --json for analysis.

  python tools/tune.py --sets conv,sgemm-full --out boda-1_amd/tuning/gfx950.tune
"""
import argparse
import re
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)

import boda_hip  # noqa: E402
from boda_hip import ops, runner  # noqa: E402

SETS = {"sgemm-full": "sgemm-ops-full.txt", "sgemm-small": "sgemm-ops-small.txt",
        "conv": "conv-ops-1-5-20-nin-alex-gn.txt", "op-sigs": "op_sigs_full.txt",
        # the conv / fc shapes of the five reference nets at batch 20 (tools/net_ops.py)
        "nets": os.path.join(ROOT, "boda-1_amd", "tuning", "net-ops-b20.txt"),
        "nets-b1": os.path.join(ROOT, "boda-1_amd", "tuning", "net-ops-b1.txt"),
        "nets-b5": os.path.join(ROOT, "boda-1_amd", "tuning", "net-ops-b5.txt")}
SPLITS = [1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 32, 48, 64]
CFG_BK = {}


def bk_of(name):
    """K tile depth of a config name like 128x128x32 or sk32x32x64w8."""
    if name.startswith(("dc", "dm", "fcv", "ks", "kn", "kd", "kw", "kr", "wg", "wx")):
        return 1 << 30
    if name.startswith("gv"):
        m = re.search(r"w(\d+)", name)
        return 16 * (int(m.group(1)) if m else 4)
    return int(re.match(r"\d+", name.split("x")[2]).group(0))


FLUSH = None

# Winograd candidates are admitted only inside Boda's Winograd tolerance: the element-wise
# min_sig_mag_rel_diff(1, ., .) against the double-accumulated oracle <= WINO_TOL, the reference's
# widening for cuDNN's 3x3 Winograd (src/rtc_prof.cc:314-319). Checked on the whole output up to
# GATE_FULL_FLOPS (as tests/test_gpu_routed.py checks it), above that on GATE_SAMPLES outputs at
# GATE_MARGIN of the tolerance (a sample's maximum understates the tensor's).
WINO_TOL = 2e-3
GATE_FULL_FLOPS = 2e10
GATE_SAMPLES = 1 << 18
GATE_MARGIN = 0.8
_REF = {}


def wino_error(wl, s, i=0):
    """Max element metric of op i's current output (the route just run) against the oracle."""
    import numpy as np
    from oracle import oracle as orc
    key = tuple(s.as_dims())
    if key not in _REF:
        inp, filts, biases = orc.gen_conv(s, 5)
        n = s.B * s.OC * s.OH * s.OW
        if n <= GATE_SAMPLES or s.flops() <= GATE_FULL_FLOPS:
            _REF[key] = (None, orc.conv_ref(inp, filts, biases, s, 1))
        else:
            idx = np.random.default_rng(5).choice(n, GATE_SAMPLES, replace=False).astype(np.uint64)
            _REF[key] = (idx.astype(np.int64), orc.conv_ref_at(inp, filts, biases, s, idx, 1))
    idx, ref = _REF[key]
    wl.launch(i)
    got = wl.output(i)
    if idx is not None:
        got = got[idx]
    return orc.normalized_errors(ref, got)[2] / (1.0 if idx is None else GATE_MARGIN)


TIMING = "graph"


def time_op(dev, wl, i, reps):
    """GPU ms per call in the regime the bench reports (TIMING "graph"): amortized over a
    replayed hipGraph of back-to-back calls (runner.op_graph_time). TIMING "flush": see
    time_op_flush."""
    if TIMING == "flush":
        return time_op_flush(dev, wl, i, reps)
    wl.launch(i)  # warm-up (grows the split-K workspace)
    b, e = dev.time_next_call()
    wl.launch(i)
    dev.sync()
    est = dev.elapsed_ms(b, e) * 1e-3
    dev.events_reset()
    n = max(3, min(100, int(round(1e-3 / max(est, 1e-6)))))
    t = min(wl.op_graph_time(i, n) for _ in range(2))
    dev.events_reset()
    return t * 1e3


def time_op_flush(dev, wl, i, reps):
    """Median GPU time of one call (ms) as the bench sees it: each launch preceded by a
    512 MiB memset that evicts L2 and the Infinity Cache (in the bench every op runs after
    220 others), timed by events on the call's own kernel dispatches."""
    global FLUSH
    if FLUSH is None:
        FLUSH = dev.alloc(512 << 20)
    wl.launch(i)  # warm-up (grows the split-K workspace)
    ev = []
    for _ in range(reps):
        FLUSH.zero()
        b, e = dev.time_next_call()
        wl.launch(i)
        ev.append((b, e))
    dev.sync()
    out = [dev.elapsed_ms(b, e) for b, e in ev]
    dev.events_reset()
    return statistics.median(out)


def pick_route(med, err, prev, rejected, min_gain):
    """The route a confirmed sweep writes for one op.

    med: {(cfg, splits): median ms}, ("default", 0) = the heuristic route (table off); err: {(cfg,
    splits): element error vs the oracle} (min_sig_mag_rel_diff(1), routes without a measurement absent);
    prev: the --out table's route or None; rejected: routes over their accuracy gate (never chosen).
    Returns (cfg, splits) or None = no table entry (the default route is at least as good).
      * the fastest admissible route, but the previous table route stays unless beaten by min_gain;
      * among the routes within min_gain of that pick, the most accurate one (an element error
        measured lower by at least 2x) -- two routes that time alike should not differ 3x in error
        (dm3 at 6e-4 where gvs gives 2e-4 on the same op);
      * a previous route that is rejected never survives, and when the default wins the op gets no
        entry (write_table then DELETES a merged table's old line)."""
    ok = {r: t for r, t in med.items() if r not in rejected}
    if not ok:
        return None
    r_best = min(ok, key=lambda r: ok[r])
    t_best = ok[r_best]
    if prev is not None and prev in ok and prev != r_best and t_best >= (1 - min_gain) * ok[prev]:
        r_best, t_best = prev, ok[prev]
    e_best = err.get(r_best)
    if e_best is not None:
        near = [r for r, t in ok.items() if t <= t_best / (1 - min_gain) and r in err and 2 * err[r] <= e_best]
        if near:
            r_best = min(near, key=lambda r: (err[r], ok[r]))
    return None if r_best[0] == "default" else r_best


def write_table(args, plat, table, results):
    """table: {key: (cfg, splits, ms, default ms, wt)}, or {key: None} = the op must have no entry
    (with --merge its old line is removed)."""
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    lines = {k: "%s cfg=%s splits=%d red=%s%s" % (k, v[0], abs(v[1]), "k" if v[1] < 0 else "i", " wt=1" if v[4] else "")
             for k, v in table.items() if v is not None}
    if args.merge and os.path.exists(args.out):
        old = {}
        for l in open(args.out):
            if l.startswith("#") or " cfg=" not in l:
                continue
            old[l[:l.index(" cfg=")]] = l.rstrip("\n")
        old.update(lines)
        for k, v in table.items():
            if v is None:
                old.pop(k, None)
        lines = old
    tmp = args.out + ".tmp"
    with open(tmp, "w") as f:
        f.write("# boda-1_amd tuning table (tools/tune.py) for %s; <op> <dims> cfg=<tile config> splits=<K splits>\n"
                % plat)
        for k in sorted(lines, key=lambda k: (k.split()[0], [int(x) for x in k.split()[1:]])):
            f.write(lines[k] + "\n")
    os.replace(tmp, args.out)
    if args.json:
        json.dump({"plat": plat, "results": results}, open(args.json, "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="conv,sgemm-full,sgemm-small")
    ap.add_argument("--out", default=os.path.join(ROOT, "boda-1_amd", "tuning", "gfx950.tune"))
    ap.add_argument("--json", default="")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--timing", choices=["graph", "flush"], default="graph")
    ap.add_argument("--max-flop-sgemm", type=float, default=3e12, help="skip sgemm sweeps above this (use heuristic)")
    ap.add_argument("--merge", action="store_true", help="keep --out entries of ops not swept in this run")
    ap.add_argument("--min-gain", type=float, default=0.03, help="with --cfg-re: replace the table's choice "
                    "only if the new best is this much faster (timings vary a few %% from box to box)")
    ap.add_argument("--cfg-re", default="", help="sweep only configs matching this regex (plus the --out "
                    "table's current choice for the op, timed again, so the better one is kept)")
    ap.add_argument("--max-splits", type=int, default=64, help="largest K split count to sweep")
    ap.add_argument("--key-re", default="", help="sweep only ops whose table key ('conv B IC H W ...') matches")
    ap.add_argument("--only-untuned", action="store_true", help="sweep only ops the --out table has no entry "
                    "for (use with --merge)")
    ap.add_argument("--wt", choices=["try", "off", "only"], default="try",
                    help="output store policy: try write-through (wt=1) on each op's best config and keep it if "
                         "faster by --wt-gain; 'only': keep the --out table's configs, sweep just the policy")
    ap.add_argument("--wt-gain", type=float, default=0.01)
    ap.add_argument("--confirm", type=int, default=0, help="re-time the TOP fastest routes of the sweep (and the "
                    "--out table's current choice) this many times each and pick by median: one timing per "
                    "candidate picks the luckiest of many noisy draws")
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--keep-prev", action="store_true", help="load the --out table's choices as with --cfg-re: "
                    "kept unless beaten by --min-gain")
    args = ap.parse_args()
    # tune against the built-in heuristic, not against a previously committed table (set here, not at
    # import: importing this module -- tests/test_tune_cpu.py, tools/cfgprobe.py -- must not change the
    # route of every later call in the importing process; the table loads at the first conv / sgemm call)
    os.environ["BH_TUNE_FILE"] = "/nonexistent"
    global TIMING
    TIMING = args.timing

    dev = boda_hip.Device(0)
    plat = dev.plat_tag()
    names = {0: boda_hip.tune_cfg_names(0), 1: boda_hip.tune_cfg_names(1)}
    table, results = {}, []
    prev = {}
    if (args.cfg_re or args.wt == "only" or args.keep_prev) and os.path.exists(args.out):
        for l in open(args.out):
            m = re.match(r"(.*) cfg=(\S+) splits=(\d+) red=(\w)", l)
            if m:
                prev[m.group(1)] = (m.group(2), int(m.group(3)) * (-1 if m.group(4) == "k" else 1))
    have = set()
    if args.only_untuned and os.path.exists(args.out):
        have = {l[:l.index(" cfg=")] for l in open(args.out) if " cfg=" in l and not l.startswith("#")}
    t_start = time.time()
    for sname in args.sets.split(","):
        o, _ = ops.read_ops(os.path.join(ROOT, "tests", "golden", "ops", SETS[sname]))  # (absolute: as is)
        shapes = []
        for op in o:
            s = ops.shape_of(op)
            if s not in shapes:
                shapes.append(s)
        for s in shapes:
            kind = 0 if isinstance(s, ops.SgemmShape) else 1
            dims = [s.M, s.N, s.K] if kind == 0 else s.as_dims()
            key = ("sgemm " if kind == 0 else "conv ") + " ".join(map(str, dims))
            if key in table or key in have or (args.key_re and not re.search(args.key_re, key)):
                continue
            wl = runner.Workload(dev, [s])
            M, N, K = (s.M, s.N, s.K) if kind == 0 else (s.OC, s.B * s.OH * s.OW, s.K)
            dev.tune_set(kind, -1, 0)
            t_def = time_op(dev, wl, 0, args.reps)
            best = (t_def, -1, 0)
            cand = []
            if not (kind == 0 and s.flops() > args.max_flop_sgemm):
                for ci, cn in enumerate(names[kind]):
                    if (args.cfg_re and not re.search(args.cfg_re, cn)) or cn == "ref64":
                        continue  # (ref64: the double-accumulating known-good kernel, never routed)
                    nkt = -(-K // bk_of(cn))
                    if cn.startswith("dm"):  # multi-channel direct conv: S = grid mode as stream-K
                        if kind == 1 and cn.startswith("dm%d" % s.KY) and s.KX == s.KY and s.sy == s.sx == 1:
                            cand += [(ci, 1), (ci, 2), (ci, 3), (ci, 5), (ci, 6)]
                        continue
                    if cn.startswith("dc"):  # direct conv (stems): no K split; UNSUP for other kernels
                        if kind == 1 and cn.startswith("dc%ds%d" % (s.KY, s.sy)) and s.KX == s.KY and s.sx == s.sy:
                            cand.append((ci, 0))
                        continue
                    if cn.startswith("wg"):  # Winograd 3x3: S = grid mode as stream-K; UNSUP for other ops
                        if kind == 1 and s.KY == s.KX == 3 and s.sy == s.sx == 1 and s.py <= 1 and s.px <= 1:
                            cand += [(ci, 1), (ci, 5), (ci, 11), (ci, 15), (ci, 21), (ci, 31)]  # one block per CU (256 AGPRs); +20: combine kernel
                        continue
                    if cn.startswith("wx"):  # position-split Winograd (planned grid); UNSUP for other ops
                        r = 5 if cn.startswith("wx25") else 3
                        if kind == 1 and s.KY == s.KX == r and s.sy == s.sx == 1 and s.py == s.px <= r // 2:
                            cand.append((ci, 0))
                            if cn.endswith("k"):  # stream-K: + the separate combine kernel (splits 20)
                                cand.append((ci, 20))
                        continue
                    if cn.startswith(("ks", "kn", "kd", "kw", "kr")):  # resident-bank 1x1: S = blocks per CU; UNSUP for other ops
                        if kind == 1 and s.KY == s.KX == 1 and s.sy == s.sx == 1 and s.py == s.px == 0:
                            cand += [(ci, 1), (ci, 2), (ci, 8)]  # 8: one unit per wave
                        continue
                    if cn.startswith("fcv"):  # batch-streaming ipconv: no K split; UNSUP for other ops
                        cand.append((ci, 0))
                        continue
                    if cn.startswith("srk"):  # stream-K: S = blocks per CU
                        cand += [(ci, 1), (ci, 2), (ci, 5), (ci, 6)]  # 5, 6: whole tiles per block
                        continue
                    if cn.startswith("gv"):  # register-streaming kernels: S = K chunks
                        tm, tn = map(int, re.match(r"gv[pqso]?(\d+)x(\d+)", cn).groups())
                        tiles = -(-M // tm) * -(-N // tn)
                        if tiles <= 512:
                            cand += [(ci, S) for S in [0] + SPLITS if S == 0 or nkt >= S]
                        continue
                    for S in SPLITS:
                        if (S > 1 and nkt < 2 * S) or S > args.max_splits:
                            continue
                        cand.append((ci, S))
                        if S > 1:
                            cand.append((ci, -S))  # same split, separate reduce kernel
            if args.wt == "only":
                cand = []
            if key in prev and prev[key][0] in names[kind]:
                cand.append((names[kind].index(prev[key][0]), prev[key][1]))
            rejected = set()
            for ci, S in cand:
                dev.tune_set(kind, ci, S)
                try:
                    t = time_op(dev, wl, 0, args.reps)
                except boda_hip.UnsupportedError:
                    continue
                if names[kind][ci].startswith(("wg", "wx")):
                    err = wino_error(wl, s)
                    if err > WINO_TOL:  # outside the Winograd tolerance: never routed
                        results.append({"key": key, "cfg": names[kind][ci], "splits": S, "ms": t, "rejected": err})
                        rejected.add((names[kind][ci], S))
                        continue
                results.append({"key": key, "cfg": names[kind][ci], "splits": S, "ms": t})
                if t > 5.0:  # long ops: a progress line per candidate (a silent minute reads as a hang)
                    print("   %s S=%+d %.4f ms" % (names[kind][ci], S, t), flush=True)
                if t < best[0]:
                    best = (t, ci, S)
            dev.tune_set(kind, -1, 0)
            results.append({"key": key, "cfg": "default", "splits": 0, "ms": t_def})
            if args.confirm > 0:
                # the TOP routes of the sweep and the table's choice, timed again: medians decide
                mine = sorted([x for x in results if x["key"] == key and x["cfg"] != "default" and "wt" not in x
                               and "rejected" not in x], key=lambda x: x["ms"])
                fin, seen = [], set()
                for x in mine:
                    k2 = (x["cfg"], x["splits"])
                    if k2 not in seen and len(fin) < args.top:
                        seen.add(k2)
                        fin.append(k2)
                if (key in prev and prev[key] not in seen and prev[key][0] in names[kind]
                        and prev[key] not in rejected):
                    fin.append(prev[key])
                # the default route (table off: the heuristic) competes too, so a confirmed route
                # slower than it is never written
                dev.tune_set(kind, -1, 0)
                med = {("default", 0): statistics.median(time_op(dev, wl, 0, args.reps) for _ in range(args.confirm))}
                errs = {}
                if kind == 1:  # every finalist's element error (the most accurate of near-equal routes wins)
                    errs[("default", 0)] = wino_error(wl, s)
                for cn, S in fin:
                    dev.tune_set(kind, names[kind].index(cn), S)
                    try:
                        med[(cn, S)] = statistics.median(time_op(dev, wl, 0, args.reps) for _ in range(args.confirm))
                        if kind == 1:
                            errs[(cn, S)] = wino_error(wl, s)
                    except boda_hip.UnsupportedError:
                        pass
                dev.tune_set(kind, -1, 0)
                for (cn, S), t in med.items():
                    results.append({"key": key, "cfg": cn, "splits": S, "ms": t, "confirm": args.confirm,
                                    "err": errs.get((cn, S))})
                pick = pick_route(med, errs, prev.get(key), rejected, args.min_gain)
                best = (t_def, -1, 0) if pick is None else (med[pick], names[kind].index(pick[0]), pick[1])
            elif key in prev and prev[key] not in rejected:  # keep the table's choice unless clearly beaten
                pt = [x["ms"] for x in results if x["key"] == key and x["cfg"] == prev[key][0]
                      and x["splits"] == prev[key][1]]
                if pt and best[0] >= (1 - args.min_gain) * pt[0]:
                    best = (pt[0], names[kind].index(prev[key][0]), prev[key][1])
            wt = 0
            if best[1] >= 0 and args.wt != "off":
                # the same route with write-through output stores (bit-identical results)
                dev.tune_set(kind, best[1], best[2])
                dev.tune_set_policy(kind, 1)
                try:
                    t = time_op(dev, wl, 0, args.reps)
                    dev.tune_set_policy(kind, 0)
                    t0 = time_op(dev, wl, 0, args.reps)  # the same route timed again, write-back
                    results.append({"key": key, "cfg": names[kind][best[1]], "splits": best[2], "wt": 1, "ms": t,
                                    "ms_wb": t0})
                    if t < (1 - args.wt_gain) * min(t0, best[0]):
                        best, wt = (t, best[1], best[2]), 1
                except boda_hip.UnsupportedError:
                    pass
                dev.tune_set_policy(kind, -1)
                dev.tune_set(kind, -1, 0)
            wl.free()
            # no route beats the default (or the previous entry was rejected): no entry, and a merged
            # table's old line for the op is deleted
            table[key] = (names[kind][best[1]], best[2], best[0], t_def, wt) if best[1] >= 0 else None
            rf = runner.roofline_secs(s) * 1e3
            print("%-48s default %.4f ms  best %s S=%+d %.4f ms  roofline %.4f ms (%.0f%%)" % (
                key, t_def, names[kind][best[1]] if best[1] >= 0 else "default", best[2], best[0], rf,
                100 * rf / best[0]), flush=True)
            if args.merge:  # written after every op: a sweep cut short by a time limit keeps its progress
                write_table(args, plat, table, results)
    write_table(args, plat, table, results)
    print("wrote %d entries (%d deletions) to %s in %.0f s" % (sum(v is not None for v in table.values()),
                                                          sum(v is None for v in table.values()), args.out,
                                                          time.time() - t_start))
    dev.close()


if __name__ == "__main__":
    main()
