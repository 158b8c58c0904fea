#!/usr/bin/env python3
"""Decode the reference's known-good digests into committed JSON fixtures.

Run ONCE in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It reads only DATA files of the reference:
  * test/good_tr/<suite>/wisdom.wis  -- text stream of op_wisdom_t blocks whose
    'kg' entries are hex-encoded binary nda digests (format: src/op-tuner.cc:68-140,
    digest layout src/boda_base.cc:330-338, dims layout src/boda_base.H:728-746);
  * test/*.txt op lists (copied verbatim into tests/golden/ops/ as input data).

Output: tests/golden/<suite>.json = [{"op": <op line>, "kgs": [{"var", "tn",
"self_cmp_mrd", "dims": [[name, sz, stride], ...], "strides_sz", "seed",
"min", "max", "samps": [...]}]}] with floats stored as IEEE-754 hex words so
they round-trip bit-exactly. Nothing here runs or imports reference code.
"""
import json
import os
import shutil
import struct
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

SUITES = ["sgemm-gen600", "sgemm-gen5", "conv-gen5", "conv-debug", "conv-full-gen5",
          "ops-prof-conv-3x3-cudnn-boda"]
OP_LISTS = ["sgemm-ops-tiny.txt", "sgemm-ops-small.txt", "sgemm-ops-full.txt", "sgemm-ops-debug.txt",
            "sgemm-ops-micro.txt", "conv-ops-1-5-20-nin-alex-gn.txt", "conv-ops-debug.txt",
            "conv-ops-debug-tmp.txt", "conv-ops-tiny.txt", "conv-ops-small.txt", "op_sigs_full.txt",
            "op_sigs.txt"]


class Rd:
    def __init__(self, b):
        self.b, self.o = b, 0

    def take(self, fmt):
        v = struct.unpack_from("<" + fmt, self.b, self.o)
        self.o += struct.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def string(self):
        n = self.take("I")
        s = self.b[self.o:self.o + n].decode()
        self.o += n
        return s


def f32hex(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def decode_digest(hexstr):
    r = Rd(bytes.fromhex(hexstr))
    nonnull = r.take("B")
    assert nonnull == 1
    tn = r.string()
    assert tn == "float", tn
    magic = r.take("I")
    assert magic == 0xDADA0101, hex(magic)
    self_cmp_mrd = r.take("d")
    nd = r.take("I")
    dims = []
    for _ in range(nd):
        sz, stride = r.take("I"), r.take("I")
        dims.append([r.string(), sz, stride])
    dtn = r.string()
    strides_sz = r.take("Q")
    valid = r.take("B")
    seed = r.take("Q")
    mn, mx = r.take("f"), r.take("f")
    ns = r.take("I")
    samps = [r.take("f") for _ in range(ns)]
    assert r.o == len(r.b), (r.o, len(r.b))
    return {"tn": dtn, "self_cmp_mrd": self_cmp_mrd, "dims": dims, "strides_sz": strides_sz,
            "strides_valid": valid, "seed": seed, "min": f32hex(mn), "max": f32hex(mx),
            "samps": [f32hex(s) for s in samps]}


def decode_wisdom(path):
    lines = open(path).read().split("\n")
    i, out = 0, []
    while i < len(lines):
        if lines[i] != "op_wisdom_t":
            i += 1
            continue
        ent = {"op": lines[i + 1], "kgs": []}
        i += 2
        while lines[i] != "/op_wisdom_t":
            if lines[i] == "kg":
                d = decode_digest(lines[i + 2])
                d["var"] = lines[i + 1]
                ent["kgs"].append(d)
                i += 3
            else:
                i += 1  # op_tune_wisdom_t runs are not needed for parity
        out.append(ent)
        i += 1
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are already committed")
    for s in SUITES:
        ents = decode_wisdom(os.path.join(REF, "test/good_tr", s, "wisdom.wis"))
        with open(os.path.join(HERE, s + ".json"), "w") as f:
            json.dump(ents, f, separators=(",", ":"))
        print(s, len(ents), "ops")
    os.makedirs(os.path.join(HERE, "wis"), exist_ok=True)
    for s in SUITES:  # the original text files too, for the C++ wisdom reader's round-trip test
        shutil.copyfile(os.path.join(REF, "test/good_tr", s, "wisdom.wis"), os.path.join(HERE, "wis", s + ".wis"))
    os.makedirs(os.path.join(HERE, "ops"), exist_ok=True)
    for o in OP_LISTS:
        shutil.copyfile(os.path.join(REF, "test", o), os.path.join(HERE, "ops", o))
    print("copied", len(OP_LISTS), "op lists")


if __name__ == "__main__":
    main()
