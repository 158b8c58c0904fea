#!/usr/bin/env python3
"""Per-kernel instruction mix of a hipcc -S output (loop body = the block that holds the
most v_mfma): counts of MFMA / VALU / SALU / DMA / vmcnt(0) waits, VGPRs, scratch.
  python tools/asmstat.py build/x.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = {m.group(1): m.group(0) for m in re.finditer(r"\.name:\s+(\S+)[\s\S]*?(?=\n  - \.|\Z)", s)}
for m in re.finditer(r"^(_Z\S*):", s, re.M):
    n = m.group(1)
    if pat not in n:
        continue
    i = m.end()
    j = s.index(".Lfunc_end", i)
    body = s[i:j]
    blocks = re.split(r"\n(?=\.LBB)", body)
    loop = max(blocks, key=lambda b: b.count("v_mfma"))
    def cnt(b):
        return dict(mfma=b.count("v_mfma"), valu=len(re.findall(r"^\s+v_(?!mfma)", b, re.M)),
                    salu=len(re.findall(r"^\s+s_(?!waitcnt|barrier|nop|cbranch|branch|endpgm|setprio)", b, re.M)),
                    dma=len(re.findall(r"buffer_load\S*.*\blds\b", b)), ds_read=len(re.findall(r"ds_read", b)),
                    vm0=b.count("vmcnt(0)"))
    seg = s[j:j + 3000]
    vg = re.search(r"\.vgpr_count:\s+(\d+)", s[s.find(".name:           " + n):][:4000] if ".name:           " + n in s else "")
    sc = re.search(r"; ScratchSize: (\d+)", seg)
    nv = re.search(r"; NumVgprs: (\d+)", seg)
    print(n[:100])
    print("   whole:", cnt(body), " vgpr", nv.group(1) if nv else "?", "scratch", sc.group(1) if sc else "?")
    print("   loop :", cnt(loop))
