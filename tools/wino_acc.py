"""fp32 error model of the 6x6 Winograd forms (bh_wgx.hip), for choosing interpolation points.

Simulates the kernel's arithmetic in numpy: U = G g G^T made in double and rounded once (wx_pack), V =
B^T d B in fp32 (row pass then column pass, each output a chain of fp32 FMAs), M = sum over input
channels of U * V accumulated in fp32 in channel order (the MFMA chain), Y = A^T M A in fp32, + bias,
ReLU. Compares against the double-accumulated direct conv with Boda's element metric
min_sig_mag_rel_diff(1, ., .) (src/boda_base.cc:140-153) and the normalized max used by the tests.

A point set {p_1 .. p_{a-1}} plus infinity defines (Toom-Cook, Lavin & Gray 2016):
  A^T[j][i] = p_i^j (infinity column: 1 in the last row), G[i][k] = p_i^k / prod_{l != i} (p_i - p_l)
  (infinity row: 1 at k = r - 1), B^T row i = ascending coefficients of prod_{l != i} (x - p_l), last
  row = those of prod_l (x - p_l).
Row scalings by powers of two are exact; the per-row scale s_i moves 1/s_i into G (made in double).

Usage: python tools/wino_acc.py [--op B,IC,H,W,OC,R,pad] [--imgs n] [--oc n]
Tool only (imports the oracle for the data and the reference); never on the product path.
"""
import argparse
import itertools
import os
import sys
from fractions import Fraction

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as orc  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "boda-1_amd"))
from boda_hip import ops  # noqa: E402


def polymul(a, b):
    r = [Fraction(0)] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            r[i + j] += x * y
    return r


def matrices(pts, m, r):
    """A^T (m x a), G (a x r), B^T (a x a) as Fractions for finite points pts (+ infinity)."""
    pts = [Fraction(p) for p in pts]
    a = len(pts) + 1
    assert a == m + r - 1
    AT = [[p ** j for p in pts] + [Fraction(1 if j == m - 1 else 0)] for j in range(m)]
    G = []
    for i, p in enumerate(pts):
        den = Fraction(1)
        for l, q in enumerate(pts):
            if l != i:
                den *= p - q
        G.append([p ** k / den for k in range(r)])
    G.append([Fraction(1 if k == r - 1 else 0) for k in range(r)])
    BT = []
    for i in range(len(pts)):
        poly = [Fraction(1)]
        for l, q in enumerate(pts):
            if l != i:
                poly = polymul(poly, [-q, Fraction(1)])
        BT.append(poly + [Fraction(0)])
    poly = [Fraction(1)]
    for q in pts:
        poly = polymul(poly, [-q, Fraction(1)])
    BT.append(poly)
    return AT, G, BT


def scale_rows(AT, G, BT):
    """Scale each B^T row by a power of two so its largest coefficient is in [1, 2) -- exact in fp32,
    the inverse goes into G (double). Likewise A^T columns: the scale moves into G's rows."""
    BT2, G2 = [row[:] for row in BT], [row[:] for row in G]
    for i, row in enumerate(BT):
        mx = max(abs(x) for x in row)
        e = 0
        while mx * Fraction(2) ** e >= 2:
            e -= 1
        while mx * Fraction(2) ** e < 1:
            e += 1
        s = Fraction(2) ** e
        BT2[i] = [x * s for x in row]
        G2[i] = [x / s for x in G2[i]]
    AT2 = [row[:] for row in AT]
    a = len(G)
    for i in range(a):
        mx = max(abs(AT[j][i]) for j in range(len(AT)))
        e = 0
        while mx * Fraction(2) ** e > 1:
            e -= 1
        while mx * Fraction(2) ** e <= Fraction(1, 2):
            e += 1
        s = Fraction(2) ** e
        for j in range(len(AT)):
            AT2[j][i] = AT[j][i] * s
        G2[i] = [x / s for x in G2[i]]
    return AT2, G2, BT2


def check_identity(AT, G, BT, m, r):
    """y = A^T [(G g) . (B^T d)] is the correlation of d (length m + r - 1) with g (length r)."""
    rng = np.random.default_rng(1)
    d = rng.standard_normal(m + r - 1)
    g = rng.standard_normal(r)
    y = np.array(AT, float) @ ((np.array(G, float) @ g) * (np.array(BT, float) @ d))
    ref = np.array([d[j:j + r] @ g for j in range(m)])
    return float(np.max(np.abs(y - ref)))


def fma_chain(coefs, xs):
    """sum_k c_k x_k as the kernel's fp32 FMA chain: nonzero terms, +-1 terms added, others fma'd."""
    acc = None
    for c, x in zip(coefs, xs):
        if c == 0:
            continue
        cf = np.float32(float(c))
        if acc is None:
            acc = (cf * x).astype(np.float32) if c not in (1, -1) else (x if c == 1 else -x)
        else:
            acc = (np.float64(cf) * x.astype(np.float64) + acc.astype(np.float64)).astype(np.float32)
    return acc if acc is not None else np.zeros_like(xs[0])


def f32(v):
    return np.float32(float(v))


def fma(a, x, y):
    """fp32 fmaf(a, x, y) with a scalar coefficient a (rounded to fp32 first)."""
    return (np.float64(f32(a)) * x.astype(np.float64) + y.astype(np.float64)).astype(np.float32)


def bt_sym(x, p, q):
    """The kernel's factored B^T for {0, p, -p, q, -q, inf} (bh_wgx.hip bt6): x is a list of 6 fp32 arrays."""
    p2, q2 = p * p, q * q
    u, v = fma(-q2, x[2], x[4]), fma(-q2, x[1], x[3])
    uu, vv = fma(-p2, x[2], x[4]), fma(-p2, x[1], x[3])
    return [fma(p2 * q2, x[0], fma(-(p2 + q2), x[2], x[4])), fma(p, v, u), fma(-p, v, u),
            fma(q, vv, uu), fma(-q, vv, uu), fma(p2 * q2, x[1], fma(-(p2 + q2), x[3], x[5]))]


def at_sym(x, p, q, m):
    """A^T for {0, p, -p, q, -q, inf}, m = 4 or 2 output rows."""
    s1, d1 = (x[1] + x[2]).astype(np.float32), (x[1] - x[2]).astype(np.float32)
    s2, d2 = (x[3] + x[4]).astype(np.float32), (x[3] - x[4]).astype(np.float32)
    y0 = ((x[0] + s1).astype(np.float32) + s2).astype(np.float32)
    if m == 2:
        return [y0, (fma(q, d2, (f32(p) * d1).astype(np.float32)) + x[5]).astype(np.float32)]
    return [y0, fma(q, d2, (f32(p) * d1).astype(np.float32)), fma(q * q, s2, (f32(p * p) * s1).astype(np.float32)),
            (fma(q ** 3, d2, (f32(p ** 3) * d1).astype(np.float32)) + x[5]).astype(np.float32)]


def transform2_fn(fn, X):
    rows = fn([X[..., j, :] for j in range(X.shape[-2])])
    Y = np.stack(rows, axis=-2)
    cols = fn([Y[..., :, j] for j in range(Y.shape[-1])])
    return np.stack(cols, axis=-1)


def transform2(T, X, exact):
    """T X T^T on the last two axes of X (rows, then columns)."""
    a = len(T)
    if exact:
        Tm = np.array(T, float)
        return np.einsum("ij,...jk,lk->...il", Tm, X.astype(np.float64), Tm)
    rows = [fma_chain(T[i], [X[..., j, :] for j in range(X.shape[-2])]) for i in range(a)]
    Y = np.stack(rows, axis=-2)
    cols = [fma_chain(T[i], [Y[..., :, j] for j in range(Y.shape[-1])]) for i in range(a)]
    return np.stack(cols, axis=-1)


def simulate(inp, filts, bias, s, m, AT, G, BT, exact=(), sym=None):
    r = s.KY
    a = m + r - 1
    B, IC, H, W, OC, pad = s.B, s.IC, s.H, s.W, s.OC, s.py
    OH, OW = H + 2 * pad - r + 1, W + 2 * pad - r + 1
    TH, TW = -(-OH // m), -(-OW // m)
    x = inp.reshape(B, IC, H, W)
    xp = np.zeros((B, IC, TH * m + r - 1, TW * m + r - 1), np.float32)
    xp[:, :, pad:pad + H, pad:pad + W] = x
    # patches [B, IC, TH, TW, a, a]
    idx_y = (np.arange(TH) * m)[:, None] + np.arange(a)[None, :]
    idx_x = (np.arange(TW) * m)[:, None] + np.arange(a)[None, :]
    d = xp[:, :, idx_y[:, None, :, None], idx_x[None, :, None, :]]
    V = transform2_fn(lambda x: bt_sym(x, *sym), d) if sym else transform2(BT, d, "V" in exact)
    V = V.astype(np.float64 if "V" in exact else np.float32)
    f = filts.reshape(OC, IC, r, r).astype(np.float64)
    Gm = np.array(G, float)
    U = np.einsum("ij,ocjk,lk->ocil", Gm, f, Gm)
    if "U" not in exact:
        U = U.astype(np.float32)
    # M[B, OC, TH, TW, a, a] = sum_ic U[oc, ic] V[b, ic, ...]
    if "M" in exact:
        M = np.einsum("ocij,bctuij->botuij", U.astype(np.float64), V.astype(np.float64))
    else:
        M = np.zeros((B, OC, TH, TW, a, a), np.float32)
        for c in range(IC):
            prod = (U[None, :, c, None, None, :, :].astype(np.float32) * V[:, None, c]).astype(np.float32)
            M = (M + prod).astype(np.float32)
    Y = transform2_fn(lambda x: at_sym(x, sym[0], sym[1], m), M) if sym else transform2(AT, M, "Y" in exact)
    Y = Y.astype(np.float64 if "Y" in exact else np.float32)
    # [B, OC, TH, TW, m, m] -> [B, OC, OH, OW]
    Y = Y.transpose(0, 1, 2, 4, 3, 5).reshape(B, OC, TH * m, TW * m)[:, :, :OH, :OW]
    out = Y + bias.reshape(1, OC, 1, 1).astype(Y.dtype)
    out = np.maximum(out, 0)
    return out.astype(np.float32).reshape(-1)


def hyb(ref, got):
    r, g = ref.astype(np.float64), got.astype(np.float64)
    d = np.abs(g - r)
    return float(np.max(d / np.maximum(1.0, np.maximum(np.abs(r), np.abs(g))))), \
        float(d.max() / max(1.0, np.abs(r).max()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="20,96,27,27,256,5,2")
    ap.add_argument("--imgs", type=int, default=2)
    ap.add_argument("--oc", type=int, default=64)
    ap.add_argument("--stages", action="store_true", help="also run with one stage exact at a time")
    ap.add_argument("--sets", default="")
    ap.add_argument("--sym", default="", help="p,q;p,q;...: factored symmetric sets {0, +-p, +-q} to simulate")
    ap.add_argument("--search", type=int, default=0, help="screen all 0 + 4-point sets from a pool, print the best N")
    a = ap.parse_args()
    B, IC, H, W, OC, R, pad = map(int, a.op.split(","))
    full = ops.ConvShape(B, IC, H, W, OC, R, R, 1, 1, pad, pad)
    inp, filts, bias = orc.gen_conv(full, 5)
    nb, noc = min(a.imgs, B), min(a.oc, OC)
    inp = inp.reshape(B, IC, H * W)[:nb].reshape(-1)
    filts = filts.reshape(OC, -1)[:noc].reshape(-1)
    bias = bias[:noc]
    s = ops.ConvShape(nb, IC, H, W, noc, R, R, 1, 1, pad, pad)
    ref = orc.conv_ref(inp, filts, bias, s, 1)
    m = 6 - R + 1
    sets = {
        "0,1,-1,2,-2": [0, 1, -1, 2, -2],
        "0,1,-1,1/2,-1/2": [0, 1, -1, Fraction(1, 2), -Fraction(1, 2)],
        "0,1,-1,2,-1/2": [0, 1, -1, 2, -Fraction(1, 2)],
        "0,1,-1,1/2,-2": [0, 1, -1, Fraction(1, 2), -2],
        "0,1,-1,3/2,-3/2": [0, 1, -1, Fraction(3, 2), -Fraction(3, 2)],
        "0,1,-1,2/3,-2/3": [0, 1, -1, Fraction(2, 3), -Fraction(2, 3)],
        "0,1,-1,3/4,-3/4": [0, 1, -1, Fraction(3, 4), -Fraction(3, 4)],
        "0,2/3,-2/3,3/2,-3/2": [0, Fraction(2, 3), -Fraction(2, 3), Fraction(3, 2), -Fraction(3, 2)],
    }
    if a.search:
        # symmetric sets {0, +-p, +-q}: the input transform keeps the shared (u, v) form of the
        # standard set (12 FMAs per 6-vector), whatever p and q are
        # scale c = p and ratio r = q / p of the symmetric set, on a grid of 1/48 steps
        cands = []
        for cn in range(24, 49, 2):
            for rn in range(72, 169, 6):
                p_, q_ = Fraction(cn, 48), Fraction(cn, 48) * Fraction(rn, 48)
                cands.append([Fraction(0), p_, -p_, q_, -q_])
        cands.append([Fraction(0), Fraction(1), Fraction(-1), Fraction(2), Fraction(-2)])
        res = []
        for pts in cands:
            AT, G, BT = matrices(pts, m, R)
            got = simulate(inp, filts, bias, s, m, AT, G, BT, sym=(pts[1], pts[3]))
            d = got.astype(np.float64) - ref.astype(np.float64)
            rms = float(np.sqrt(np.mean(d * d)) / max(1.0, np.abs(ref).max()))
            res.append((rms, hyb(ref, got)[0], "p=%s q=%s (r=%.4f)" % (pts[1], pts[3], float(pts[3] / pts[1]))))
        res.sort()
        for r_ in res[:a.search]:
            print("rms %.3e  hyb %.3e  %s" % r_)
        return
    if a.sym:
        for pq in a.sym.split(";"):
            p_, q_ = (Fraction(x) for x in pq.split(","))
            pts = [Fraction(0), p_, -p_, q_, -q_]
            AT, G, BT = matrices(pts, m, R)
            got = simulate(inp, filts, bias, s, m, AT, G, BT, sym=(p_, q_))
            h, nm = hyb(ref, got)
            d = got.astype(np.float64) - ref.astype(np.float64)
            print("factored p=%s q=%s  hyb %.3e  norm %.3e  rms %.3e" % (p_, q_, h, nm, np.sqrt(np.mean(d * d)) / max(1.0, np.abs(ref).max())), flush=True)
        return
    if a.sets:
        sets = {k: v for k, v in sets.items() if k in a.sets.split(";")}
    for name, pts in sets.items():
        for scaled in (False, True):
            AT, G, BT = matrices(pts, m, R)
            if scaled:
                AT, G, BT = scale_rows(AT, G, BT)
            err_id = check_identity(AT, G, BT, m, R)
            got = simulate(inp, filts, bias, s, m, AT, G, BT)
            h, nm = hyb(ref, got)
            line = "%-18s scaled=%d id=%.1e  hyb %.3e  norm %.3e" % (name, scaled, err_id, h, nm)
            if a.stages:
                for ex in ("V", "M", "Y"):
                    h2, _ = hyb(ref, simulate(inp, filts, bias, s, m, AT, G, BT, exact=(ex,)))
                    line += "  %s-exact %.3e" % (ex, h2)
            print(line, flush=True)
            bt_max = max(abs(float(x)) for row in BT for x in row)
            at_max = max(abs(float(x)) for row in AT for x in row)
            print("   |B^T|max %.3g  |A^T|max %.3g" % (bt_max, at_max))


if __name__ == "__main__":
    main()
