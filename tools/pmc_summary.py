#!/usr/bin/env python3
"""Summarize tools/pmc.sh passes of one op (tools/profile_op.py): per-dispatch medians of every
counter for the dispatches of the kernel whose name contains --kernel, plus the ratios DESIGN quotes
(LDS bank-conflict share, MFMA busy cycles per MFMA instruction, s_waitcnt share of wave cycles,
 HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE KiB per MI355X_MICROARCH.md's gfx950 correction).

  python tools/pmc_summary.py gpurun_out/pmc1 --kernel wgp_kernel --op "conv 20 384 13 13 384 3 3 1 1 1 1" \
      --json profiles/r03/pmc_wino.json
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--op", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    per = {}  # counter -> {dispatch: value}
    name = ""
    for f in glob.glob(os.path.join(a.dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            d = per.setdefault(r["Counter_Name"], {})
            key = (f, r["Dispatch_Id"])
            d[key] = d.get(key, 0.0) + float(r["Counter_Value"])
    med = {c: statistics.median(v.values()) for c, v in sorted(per.items())}
    out = {"op": a.op, "kernel": name[:160], "dispatches": max((len(v) for v in per.values()), default=0),
           "counters_median_per_dispatch": med}
    g = lambda k: med.get(k)  # noqa: E731
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_share"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    if g("SQ_WAIT_INST_ANY") is not None and g("SQ_WAVE_CYCLES"):
        out["waitcnt_share_of_wave_cycles"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
    if g("SQ_VALU_MFMA_BUSY_CYCLES") is not None and g("SQ_INSTS_MFMA"):
        # 64 for v_mfma_f32_32x32x2_f32 (busy cycles summed over SIMDs; utilisation = these over
        # 1024 SIMDs x the kernel's cycles)
        out["mfma_busy_cycles_per_mfma_inst"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / g("SQ_INSTS_MFMA")
    if g("SQ_INSTS_MFMA"):
        out["valu_salu_per_mfma_inst"] = ((g("SQ_INSTS_VALU") or 0) + (g("SQ_INSTS_SALU") or 0)) / g("SQ_INSTS_MFMA")
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        out["hbm_bytes"] = (2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None and g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        out["l2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    s = json.dumps(out, indent=1)
    print(s)
    if a.json:
        open(a.json, "w").write(s + "\n")


if __name__ == "__main__":
    main()
