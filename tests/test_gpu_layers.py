"""GPU parity of the non-conv forward layers (bh_fwdops.hip, through the C-ABI) against the
CPU restatements in oracle/layers.py, on the layer shapes of the reference nets (AlexNet /
NiN / GoogLeNet prototxts) and ragged edge cases. Bars: max pooling, ReLU and channel copies
bit-exact; average pooling bit-exact (same fp32 summation order); LRN and softmax within
2e-6 relative (device powf / expf vs numpy: one or two ulp)."""
import numpy as np
import pytest

import boda_hip
from oracle import layers as L

pytestmark = pytest.mark.gpu


def _up(dev, x):
    b = dev.alloc_floats(x.size)
    b.upload(np.ascontiguousarray(x, dtype=np.float32))
    return b


def _rand(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


POOLS = [  # B, C, H, W, KY, KX, sy, sx, py, px, avg
    (20, 96, 55, 55, 3, 3, 2, 2, 0, 0, 0),   # AlexNet pool1
    (5, 192, 56, 56, 3, 3, 2, 2, 0, 0, 0),   # GoogLeNet pool2 (ceil rule)
    (4, 480, 14, 14, 3, 3, 1, 1, 1, 1, 0),   # GoogLeNet inception pool branch
    (3, 1024, 7, 7, 7, 7, 1, 1, 0, 0, 1),    # GoogLeNet global average pool
    (2, 7, 9, 11, 3, 2, 2, 3, 1, 1, 1),      # ragged, padded average
    (1, 3, 5, 5, 4, 4, 3, 3, 2, 2, 0),       # partial windows at both ends
    (2, 5, 40, 37, 3, 3, 1, 1, 1, 1, 1),     # wide rows: padded average, stride 1
    (2, 3, 30, 41, 2, 2, 2, 2, 0, 0, 0),     # 2x2 (VGG-style), partial last column
    (1, 2, 19, 70, 5, 4, 3, 3, 2, 1, 0),     # runtime window, partial last row
    (2, 8, 112, 112, 3, 3, 2, 2, 0, 0, 0),   # GoogLeNet pool1 plane
    (1, 4, 224, 224, 2, 2, 2, 2, 0, 0, 0),   # VGG pool1 plane
    # runtime windows: the LDS-staged kernel (bh_fwdops.hip pool_lds_kernel), its bands, plane groups
    # and the fallback
    (1, 3, 100, 100, 5, 5, 1, 1, 2, 2, 1),   # padded stride-1 average across band edges
    (1, 2, 120, 120, 5, 4, 2, 3, 2, 1, 0),   # max with argmax across band edges
    (2, 600, 6, 6, 6, 6, 1, 1, 0, 0, 1),     # global average, 2 planes per block
    (1, 1, 4, 3000, 4, 4, 2, 2, 0, 0, 0),    # rows too wide for a band: the global-memory kernel
]


@pytest.mark.parametrize("p", POOLS, ids=lambda p: "x".join(map(str, p)))
def test_pool(dev, p):
    B, C, H, W, KY, KX, sy, sx, py, px, avg = p
    x = _rand((B, C, H, W), 1)
    ref, arg = L.pool(x, KY, KX, sy, sx, py, px, avg)
    OH, OW = boda_hip.pool_out_size(H, KY, sy, py), boda_hip.pool_out_size(W, KX, sx, px)
    assert (OH, OW) == ref.shape[2:]
    dx, do, da = _up(dev, x), dev.alloc_floats(ref.size), dev.alloc_floats(ref.size)
    dev.pool(dx, do, B, C, H, W, KY, KX, sy, sx, py, px, avg, out_in_yx=da)
    np.testing.assert_array_equal(do.download().reshape(ref.shape), ref)
    if not avg:
        np.testing.assert_array_equal(da.download().reshape(ref.shape), arg)
    for b in (dx, do, da):
        b.free()


LRNS = [(20, 96, 55, 55, 5, 1e-4, 0.75, 1.0), (5, 64, 56, 56, 5, 1e-4, 0.75, 1.0), (2, 13, 3, 5, 3, 0.5, 0.6, 2.0),
        (1, 2, 4, 4, 7, 1.0, 1.0, 1.0)]


@pytest.mark.parametrize("p", LRNS, ids=lambda p: "x".join(map(str, p[:5])))
def test_lrn(dev, p):
    B, C, H, W, ls, alpha, beta, k = p
    x = _rand((B, C, H, W), 2) * 4
    ref, sb = L.lrn(x, ls, alpha, beta, k)
    dx, do, ds = _up(dev, x), dev.alloc_floats(x.size), dev.alloc_floats(x.size)
    dev.lrn(dx, do, B, C, H, W, ls, alpha, beta, k, out_scale_base=ds)
    # fma contraction, and channel chunks past the first starting their running sum fresh
    # (bh_fwdops.hip lrn_kernel; the reference sum carries +/- residue of earlier channels): < 2e-6;
    # out also carries the hardware exp2/log2 for scale^-beta (the reference's fast-math __powf)
    np.testing.assert_allclose(ds.download().reshape(x.shape), sb, rtol=2e-6, atol=0)
    np.testing.assert_allclose(do.download().reshape(x.shape), ref, rtol=2e-6, atol=1e-30)
    for b in (dx, do, ds):
        b.free()


def test_lrn_rejects_even_window(dev):
    x = dev.alloc_floats(16)
    with pytest.raises(boda_hip.UnsupportedError):
        dev.lrn(x, x, 1, 4, 2, 2, 4, 1.0, 1.0, 1.0)
    x.free()


@pytest.mark.parametrize("n", [1, 3, 4, 1000, 20 * 96 * 55 * 55 + 1])
def test_relu(dev, n):
    x = _rand((n,), 3)
    d = _up(dev, x)
    dev.relu(d, n)
    np.testing.assert_array_equal(d.download(), L.relu(x))
    d.free()


@pytest.mark.parametrize("shape", [(20, 1000, 1, 1), (2, 21, 7, 9), (1, 1, 1, 1)])
def test_softmax(dev, shape):
    x = _rand(shape, 4) * 3
    ref = L.softmax(x)
    dx, dp = _up(dev, x), dev.alloc_floats(x.size)
    dev.softmax(dx, dp, *shape)
    np.testing.assert_allclose(dp.download().reshape(shape), ref, rtol=2e-6, atol=1e-30)
    dx.free()
    dp.free()


def test_concat_and_split(dev):
    B, H, W = 3, 7, 5
    parts = [_rand((B, c, H, W), 10 + c) for c in (64, 3, 128, 32)]
    out = dev.alloc_floats(B * sum(p.shape[1] for p in parts) * H * W)
    Ct = sum(p.shape[1] for p in parts)
    oc = 0
    dps = []
    for p in parts:
        d = _up(dev, p)
        dps.append(d)
        dev.chan_copy(d, out, B, H * W, p.shape[1], 0, Ct, oc, p.shape[1])
        oc += p.shape[1]
    cat = L.concat(parts)
    np.testing.assert_array_equal(out.download().reshape(cat.shape), cat)
    # split back (split_copy.cucl: icix)
    back = dev.alloc_floats(B * 128 * H * W)
    dev.chan_copy(out, back, B, H * W, Ct, 67, 128, 0, 128)
    np.testing.assert_array_equal(back.download().reshape(B, 128, H, W), parts[2])
    for d in dps + [out, back]:
        d.free()
