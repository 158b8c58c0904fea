#!/usr/bin/env python3
"""Summarize gpurun_out/ab.log from tools/job_ab.sh: best time per op per library."""
import collections
import re
import sys

cur = key = None
res = collections.defaultdict(list)
libs = []
for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    if l.startswith("###"):
        cur = l.split()[1]
        if cur not in libs:
            libs.append(cur)
        continue
    if l.startswith("=="):
        key = l.split("roofline")[0][3:].strip()
        continue
    m = re.match(r"\s+table\s+([\d.]+) ms", l)
    if m:
        res[(key, cur)].append(float(m.group(1)) * 1e3)
keys = []
for (k, c) in res:
    if k not in keys:
        keys.append(k)
tot = [0.0] * len(libs)
for k in keys:
    b = [min(res[(k, c)]) for c in libs]
    tot = [x + y for x, y in zip(tot, b)]
    print("%-38s " % k + "  ".join("%s %7.2f" % (c[:14], x) for c, x in zip(libs, b)))
print("total " + "  ".join("%s %.1f" % (c, x) for c, x in zip(libs, tot)))
