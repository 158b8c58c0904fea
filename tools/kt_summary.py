#!/usr/bin/env python3
"""Condense tools/ktrace.py output (second repetition of each case) into phase times (us)."""
import re
import sys

cfg = shape = None
n = 0
for l in open(sys.argv[1]):
    if l.startswith('###'):
        cfg = l.strip()[4:]
        continue
    if l.startswith('=='):
        shape = l.split('variant')[0][3:].strip()
        n = 0
        continue
    if l.startswith('  post'):
        n += 1
        if n != 2:
            continue
        m = {int(k): (float(a), float(b), float(c))
             for k, a, b, c in re.findall(r'm(\d)\s+([\d.]+)/\s*([\d.]+)/\s*([\d.]+)', l)}
        post = float(l.split()[1])
        e = m[4][2] if 4 in m else m[2][2]
        print(f"{cfg:16s} {shape:32s} prol {m[1][1]-m[0][1]:5.2f} loop {m[2][1]-m[1][1]:6.2f} "
              f"tail {e-m[2][1]:5.2f} kernel(m0->end) {e-m[0][0]:6.2f} post {post:6.2f}")
