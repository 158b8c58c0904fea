"""Boda op-line parsing and per-op work model (host-side glue).

Op lines come in two dialects:
  current  (str_vals=(type=Convolution),nda_vals=(in=(dims=(img=5,...)),
            kern_sz=(tn=none,dims=(y=3,x=3)),out_chans=(tn=uint32_t,v=256),...))
           -- op_base_t{str_vals,nda_vals}, src/op_base.H:9-14
  legacy   (type=Convolution,dims_vals=(in=(img=5,...),...),str_vals=(out_chans=256))
           -- emitted by pysrc/to-prof-ops-gen.py:66-68
Both are parsed with the lexp grammar of src/lexp.cc:253-330:
  lexp := '(' [name '=' lexp {',' name '=' lexp}] ')' | leaf
(a leaf runs to the next unbalanced ')' or ','; backslash escapes).

Flop / byte model: src/latex-util.H:101-136 (conv: M = B*OY*OX, K = IC*KY*KX,
N = OC, flops = 2MNK, bytes = 4*(in + out + filts + biases); sgemm: flops = 2MNK,
bytes = 4*(MK + KN + MN)).
"""
from collections import OrderedDict
from dataclasses import dataclass, field


class LexpError(ValueError):
    pass


def parse_lexp(s):
    """Parse one lexp string into nested OrderedDicts (leaves are str)."""
    pos = 0

    def leaf():
        nonlocal pos
        out, depth = [], 0
        while pos < len(s):
            ch = s[pos]
            if ch == "\\" and pos + 1 < len(s):
                out.append(s[pos + 1])
                pos += 2
                continue
            if ch == "(":
                depth += 1
            elif ch == ")":
                if depth == 0:
                    break
                depth -= 1
            elif ch == "," and depth == 0:
                break
            out.append(ch)
            pos += 1
        return "".join(out)

    def node():
        nonlocal pos
        if pos < len(s) and s[pos] == "(":
            pos += 1
            d = OrderedDict()
            if pos < len(s) and s[pos] == ")":
                pos += 1
                return d
            while True:
                eq = s.find("=", pos)
                if eq < 0:
                    raise LexpError("expected name= at %d in %r" % (pos, s))
                name = s[pos:eq]
                if not name or any(c in name for c in "(),"):
                    raise LexpError("bad name %r at %d" % (name, pos))
                pos = eq + 1
                if name in d:
                    raise LexpError("duplicate key %r" % name)
                d[name] = node()
                if pos >= len(s):
                    raise LexpError("unterminated list in %r" % s)
                if s[pos] == ",":
                    pos += 1
                    continue
                if s[pos] == ")":
                    pos += 1
                    return d
                raise LexpError("unexpected %r at %d" % (s[pos], pos))
        return leaf()

    v = node()
    if pos != len(s):
        raise LexpError("trailing text %r" % s[pos:])
    return v


@dataclass
class Op:
    type: str
    dims: "OrderedDict[str, OrderedDict[str, int]]" = field(default_factory=OrderedDict)
    scalars: "OrderedDict[str, int]" = field(default_factory=OrderedDict)
    strs: "OrderedDict[str, str]" = field(default_factory=OrderedDict)
    line: str = ""


def _dims(d):
    out = OrderedDict()
    for k, v in d.items():
        if k == "__tn__":
            continue
        out[k] = int(v)
    return out


def parse_op(line):
    """One op line (either dialect) -> Op."""
    line = line.strip()
    t = parse_lexp(line)
    if not isinstance(t, dict):
        raise LexpError("op line is not a list: %r" % line)
    if "nda_vals" in t or ("str_vals" in t and "type" in t.get("str_vals", {})):
        sv = t.get("str_vals", OrderedDict())
        op = Op(type=sv["type"], line=line)
        for k, v in sv.items():
            if k != "type":
                op.strs[k] = v
        for name, nda in t.get("nda_vals", OrderedDict()).items():
            if "dims" in nda:
                op.dims[name] = _dims(nda["dims"])
            elif "v" in nda:
                op.scalars[name] = int(nda["v"])
        return op
    if "type" in t:  # legacy dialect
        op = Op(type=t["type"], line=line)
        for name, dd in t.get("dims_vals", OrderedDict()).items():
            op.dims[name] = _dims(dd)
        for k, v in t.get("str_vals", OrderedDict()).items():
            try:
                op.scalars[k] = int(v)
            except ValueError:
                op.strs[k] = v
        return op
    raise LexpError("unrecognised op line: %r" % line)


def conv_out_sz(i, pad, k, stride):
    """src/conv_util.cc:167-173"""
    p = i + 2 * pad
    return 0 if p < k else (p - k) // stride + 1


@dataclass(frozen=True)
class ConvShape:
    B: int
    IC: int
    H: int
    W: int
    OC: int
    KY: int
    KX: int
    sy: int
    sx: int
    py: int
    px: int

    @property
    def OH(self):
        return conv_out_sz(self.H, self.py, self.KY, self.sy)

    @property
    def OW(self):
        return conv_out_sz(self.W, self.px, self.KX, self.sx)

    @property
    def M(self):
        return self.B * self.OH * self.OW

    @property
    def K(self):
        return self.IC * self.KY * self.KX

    @property
    def N(self):
        return self.OC

    def flops(self):
        return 2 * self.M * self.N * self.K

    def bytes(self):
        return 4 * (self.B * self.IC * self.H * self.W + self.B * self.OC * self.OH * self.OW
                    + self.OC * self.K + self.OC)

    def as_dims(self):
        return [self.B, self.IC, self.H, self.W, self.OC, self.KY, self.KX, self.sy, self.sx, self.py, self.px]


@dataclass(frozen=True)
class SgemmShape:
    M: int
    N: int
    K: int

    def flops(self):
        return 2 * self.M * self.N * self.K

    def bytes(self):
        return 4 * (self.M * self.K + self.K * self.N + self.M * self.N)


def conv_shape(op):
    """Op (type Convolution) -> ConvShape, checking the reference's consistency rules."""
    if op.type != "Convolution":
        raise ValueError("not a Convolution op: %s" % op.type)
    din, df = op.dims["in"], op.dims["filts"]
    ks, st, pd = op.dims["kern_sz"], op.dims["stride"], op.dims["in_pad"]
    s = ConvShape(B=din["img"], IC=din["chan"], H=din["y"], W=din["x"], OC=df["out_chan"],
                  KY=ks["y"], KX=ks["x"], sy=st["y"], sx=st["x"], py=pd["y"], px=pd["x"])
    if df["in_chan"] != s.IC or df["y"] != s.KY or df["x"] != s.KX:
        raise ValueError("filts dims inconsistent with in / kern_sz: %s" % op.line)
    if "out" in op.dims:
        do = op.dims["out"]
        if (do["img"], do["chan"], do["y"], do["x"]) != (s.B, s.OC, s.OH, s.OW):
            raise ValueError("out dims inconsistent with conv_in_sz_to_out_sz: %s" % op.line)
    oc = op.scalars.get("out_chans")
    if oc is not None and oc != s.OC:
        raise ValueError("out_chans mismatch: %s" % op.line)
    return s


def sgemm_shape(op):
    if op.type != "sgemm":
        raise ValueError("not an sgemm op: %s" % op.type)
    a, b, c = op.dims["a"], op.dims["b"], op.dims["c"]
    s = SgemmShape(M=a["M"], N=b["N"], K=a["K"])
    if b["K"] != s.K or c["M"] != s.M or c["N"] != s.N:
        raise ValueError("sgemm dims inconsistent: %s" % op.line)
    return s


def read_ops(path, types=("Convolution", "sgemm")):
    """Read an op-list file. Returns (ops, skipped) where skipped counts lines of other types."""
    ops, skipped = [], 0
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            op = parse_op(line)
            if op.type not in types:
                skipped += 1
                continue
            ops.append(op)
    return ops, skipped


def shape_of(op):
    return conv_shape(op) if op.type == "Convolution" else sgemm_shape(op)
