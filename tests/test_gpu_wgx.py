"""Position-split Winograd kernels (bh_wgx.hip, configs wx*) against the oracle.

wx43* is F(4x4, 3x3) and wx23* F(2x2, 3x3) for stride-1 3x3 convs, wx25* F(2x2, 5x5) for stride-1
5x5 convs (square padding <= R / 2, IC % 4 == 0; the 6x6 forms also IC <= 64 / 96). They are forced with
bh_tune_set on shapes whose 32-tile units run across tile rows and images (outputs that are not a
multiple of the 4- / 2-wide tile, a last unit only partly filled), ragged output channels (not a
multiple of the 64- / 128-channel tile, nor of 32), unpadded and non-square inputs. The result is
an exact-fp32 Winograd sum, checked against the double-accumulated oracle with the tolerances of
test_gpu_conv.py and, element-wise, with Boda's Winograd tolerance: max
min_sig_mag_rel_diff(1, ref, out) <= 2e-3, what the reference allows cuDNN's 3x3 Winograd
(src/rtc_prof.cc:314-319) -- the transforms amplify fp32 cancellation on near-zero outputs, which
that metric reads as absolute error (points 0, +-2/3, +-3/2 keep the 6x6 forms inside
it). A rerun gives the same bits, a pre-packed
bank the same bits as the in-call pack, and the residual / channel-slab epilogues the plain call's
bits.
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops
from oracle import oracle as orc
from test_gpu_conv import WINO_ELEM_TOL, run_conv

pytestmark = pytest.mark.gpu

C = ops.ConvShape
WX = [n for n in boda_hip.tune_cfg_names(1) if n.startswith("wx")]

SHAPES3 = [
    C(2, 64, 13, 13, 96, 3, 3, 1, 1, 1, 1),    # odd: last tile row / column partly outside
    C(1, 32, 14, 14, 130, 3, 3, 1, 1, 1, 1),   # ragged OC (130)
    C(3, 16, 7, 7, 70, 3, 3, 1, 1, 1, 1),      # units across several images
    C(5, 24, 6, 6, 40, 3, 3, 1, 1, 1, 1),
    C(2, 8, 11, 9, 33, 3, 3, 1, 1, 1, 1),      # non-square, OC 33
    C(1, 16, 15, 15, 32, 3, 3, 1, 1, 0, 0),    # unpadded
    C(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1),
    C(1, 16, 27, 30, 64, 3, 3, 1, 1, 1, 1),
    C(2, 16, 56, 56, 64, 3, 3, 1, 1, 1, 1),    # long tile rows
    C(1, 24, 40, 62, 50, 3, 3, 1, 1, 1, 1),
    C(2, 256, 13, 13, 384, 3, 3, 1, 1, 1, 1),  # a conv-set layer (many stages)
    C(1, 512, 14, 14, 64, 3, 3, 1, 1, 1, 1),   # long K (wx23; over the 6x6 forms' cap)
    C(1, 128, 14, 14, 64, 3, 3, 1, 1, 1, 1),   # IC over F(4x4,3x3)'s cap (wx23 only)
    C(2, 64, 14, 14, 64, 3, 3, 1, 1, 1, 1),    # IC at F(4x4,3x3)'s cap
]
SHAPES5 = [
    C(2, 16, 27, 27, 96, 5, 5, 1, 1, 2, 2),    # the AlexNet conv2 geometry, odd output
    C(1, 32, 28, 28, 130, 5, 5, 1, 1, 2, 2),   # ragged OC
    C(3, 8, 7, 7, 70, 5, 5, 1, 1, 2, 2),       # units across images
    C(2, 12, 14, 14, 48, 5, 5, 1, 1, 2, 2),
    C(1, 16, 15, 17, 33, 5, 5, 1, 1, 0, 0),    # unpadded, non-square
    C(1, 8, 12, 12, 16, 5, 5, 1, 1, 1, 1),     # pad 1
    C(2, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2),   # a conv-set layer, IC at F(2x2,5x5)'s cap
]


def shapes_of(cn):
    return SHAPES5 if cn.startswith("wx25") else SHAPES3


def check(out, s):
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1)
    nm, rl2, hyb = orc.normalized_errors(ref, out)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
    assert hyb <= WINO_ELEM_TOL, (s, hyb)


@pytest.mark.parametrize("cn", WX)
def test_wx_config(dev, cn):
    ci = boda_hip.tune_cfg_names(1).index(cn)
    ran = 0
    dev.tune_set(1, ci, 0)
    try:
        for s in shapes_of(cn):
            try:
                out = run_conv(dev, s)
            except boda_hip.UnsupportedError:
                continue  # the strip does not fit this configuration's slot (another SP serves it)
            ran += 1
            check(out, s)
            np.testing.assert_array_equal(run_conv(dev, s), out)
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 3, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", [n for n in WX if n.endswith("k")])
def test_wx_combine_kernel(dev, cn):
    """Stream-K (SK 1) configurations with splits 20: the cut units summed by wx_combine_kernel after
    the grid -- the same slabs in the same block order as the last arriver, so the same bits."""
    ci = boda_hip.tune_cfg_names(1).index(cn)
    ran = 0
    try:
        for s in shapes_of(cn):
            dev.tune_set(1, ci, 0)
            try:
                out = run_conv(dev, s)
            except boda_hip.UnsupportedError:
                continue
            dev.tune_set(1, ci, 20)
            sep = run_conv(dev, s)
            check(sep, s)
            np.testing.assert_array_equal(sep, out)
            ran += 1
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 3, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", WX)
def test_wx_rejects_other_shapes(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    r = 5 if cn.startswith("wx25") else 3
    try:
        with pytest.raises(boda_hip.UnsupportedError):  # the other kernel size
            run_conv(dev, C(1, 32, 28, 28, 16, 8 - r, 8 - r, 1, 1, 1, 1))
        with pytest.raises(boda_hip.UnsupportedError):  # stride 2
            run_conv(dev, C(1, 16, 28, 28, 16, r, r, 2, 2, 1, 1))
        with pytest.raises(boda_hip.UnsupportedError):  # IC % 4 != 0
            run_conv(dev, C(1, 3, 28, 28, 16, r, r, 1, 1, 1, 1))
        with pytest.raises(boda_hip.UnsupportedError):  # pad > R / 2
            run_conv(dev, C(1, 16, 28, 28, 16, r, r, 1, 1, r, r))
        if not cn.startswith("wx23"):
            with pytest.raises(boda_hip.UnsupportedError):  # IC over the 6x6 forms' cap (element error)
                run_conv(dev, C(1, 132 if r == 3 else 100, 14, 14, 16, r, r, 1, 1, 1, 1))
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [n for n in WX if n in ("wx43s8", "wx25s6", "wx23s6")])
def test_wx_residual_and_slab(dev, cn):
    r = 5 if cn.startswith("wx25") else 3
    s = C(2, 32, 28, 28, 96, r, r, 1, 1, r // 2, r // 2)
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        plain = run_conv(dev, s, relu=0)
        n = s.B * s.OC * s.OH * s.OW
        rr = (np.random.default_rng(3).standard_normal(n) * 3).astype(np.float32)
        i, f, b = dev.alloc_floats(s.B * s.IC * s.H * s.W), dev.alloc_floats(s.OC * s.K), dev.alloc_floats(s.OC)
        dr, o = dev.alloc_floats(n), dev.alloc_floats(n)
        dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
        dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
        dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
        dr.upload(rr)
        dev.conv_res(i, f, b, dr, o, s, 1)
        exp = (plain + rr).astype(np.float32)
        np.testing.assert_array_equal(o.download(), np.where(exp < 0, np.float32(0), exp))
        ofs, ctot = 8, s.OC + 24
        so = dev.alloc_floats(s.B * ctot * s.OH * s.OW)
        so.upload(np.full(s.B * ctot * s.OH * s.OW, -7.25, np.float32))
        dev.conv_slab(i, f, b, so, ctot, ofs, s)
        got = so.download().reshape(s.B, ctot, s.OH, s.OW)
        ref = run_conv(dev, s).reshape(s.B, s.OC, s.OH, s.OW)
        np.testing.assert_array_equal(got[:, ofs:ofs + s.OC], ref)
        assert (got[:, :ofs] == -7.25).all() and (got[:, ofs + s.OC:] == -7.25).all()
        for x in (i, f, b, dr, o, so):
            x.free()
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [n for n in WX if n in ("wx43s8", "wx25s12w4", "wx23s6")])
def test_wx_dword_aligned_pointers(dev, cn):
    """Input and output pointers one float past a 16-B boundary (a caller's sub-buffer): the strip
    DMA takes any dword alignment, and the tile-row vector stores fall back to dword stores."""
    r = 5 if cn.startswith("wx25") else 3
    s = C(2, 32, 28, 28, 96, r, r, 1, 1, r // 2, r // 2)
    ni, no = s.B * s.IC * s.H * s.W, s.B * s.OC * s.OH * s.OW
    bi, bo = dev.alloc_floats(ni + 4), dev.alloc_floats(no + 4)
    f, b = dev.alloc_floats(s.OC * s.K), dev.alloc_floats(s.OC)
    vi, vo = boda_hip.DevBuf(dev, bi.ptr + 4, ni * 4), boda_hip.DevBuf(dev, bo.ptr + 4, no * 4)
    dev.gen_data(GEN_CONV_IN, vi, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        dev.conv(vi, f, b, vo, s, 1)
        got = vo.download()
        ref = run_conv(dev, s)  # the same configuration on aligned buffers
    finally:
        dev.tune_set(1, -1, 0)
    check(got, s)
    np.testing.assert_array_equal(got, ref)
    for x in (bi, bo, f, b):
        x.free()


# Shapes whose unit count leaves a partly filled last round on 256 CUs, so the split-tail grids cut
# its units into pieces (wx*t: along the stages, wx*g: by channel group): 288 F(4x4, 3x3) and 640
# F(2x2, 5x5) units of 64 channels, 8-wave blocks (one per CU)
TAIL = {
    "wx43": C(9, 8, 128, 128, 64, 3, 3, 1, 1, 1, 1),
    "wx25": C(4, 16, 64, 64, 320, 5, 5, 1, 1, 2, 2),
}


@pytest.mark.parametrize("cn", [n for n in WX if n.endswith(("t", "g"))])
def test_wx_split_tail(dev, cn):
    s = TAIL[cn[:4]]
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        out = run_conv(dev, s)
        check(out, s)
        np.testing.assert_array_equal(run_conv(dev, s), out)  # the tail pieces sum in block order
    finally:
        dev.tune_set(1, -1, 0)
