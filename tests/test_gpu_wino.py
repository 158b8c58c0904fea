"""Winograd F(2x2, 3x3) kernels (bh_wino.hip, configs wg*) against the oracle.

Each wg configuration serves stride-1 3x3 convs with pad 0 or 1 and IC % 4 == 0 (the v forms: input
widths W % 4 == 0, whose strip rows load as 16-B pieces). They are forced with bh_tune_set on
shapes whose tiles run across tile rows and images (odd 13x13 / 7x7 outputs with a half-empty last
tile row and column, 6x6, 14x14, 28x28, 56x56), ragged output channels (not a multiple of the 64- /
128-channel tile, nor of 32), unpadded and non-square inputs, under every grid mode the tuner may
pick (splits 0: stream-K at the occupancy's blocks per CU, 1 / 2 blocks per CU, 5: whole tiles per
block; 11 / 15: the same with the OC tile slowest -- the ngr fastdiv branch of tile_of and another
stream-K slab / ticket pattern; 20 / 21 / 31: the stream-K modes with the cut tiles summed by
wg_combine_kernel after the grid, bitwise equal to their last-arriver forms). The result is an exact-fp32 Winograd sum, so it is checked against the double-accumulated
oracle with the tolerances of test_gpu_conv.py -- the same bar every direct route
meets -- and element-wise within the 2e-3 the reference allows cuDNN's 3x3 Winograd
(min_sig_mag_rel_diff, src/rtc_prof.cc:314-319). A rerun gives the same bits (cut tiles are
summed in a fixed block order); a pre-packed bank gives the same bits as the in-call pack; the
residual / channel-slab epilogues equal the plain call's bits.
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops
from oracle import oracle as orc
from test_gpu_conv import WINO_ELEM_TOL, run_conv

pytestmark = pytest.mark.gpu

WG = [n for n in boda_hip.tune_cfg_names(1) if n.startswith("wg")]

SHAPES = [
    ops.ConvShape(2, 64, 13, 13, 96, 3, 3, 1, 1, 1, 1),    # odd: last tile row / column half outside
    ops.ConvShape(1, 32, 14, 14, 130, 3, 3, 1, 1, 1, 1),   # ragged OC (130)
    ops.ConvShape(3, 16, 7, 7, 70, 3, 3, 1, 1, 1, 1),      # tiles across several images
    ops.ConvShape(5, 24, 6, 6, 40, 3, 3, 1, 1, 1, 1),
    ops.ConvShape(2, 8, 11, 9, 33, 3, 3, 1, 1, 1, 1),      # non-square, OC 33
    ops.ConvShape(1, 16, 15, 15, 32, 3, 3, 1, 1, 0, 0),    # unpadded
    ops.ConvShape(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1),    # W % 4 == 0
    ops.ConvShape(1, 16, 27, 30, 64, 3, 3, 1, 1, 1, 1),
    ops.ConvShape(2, 16, 56, 56, 64, 3, 3, 1, 1, 1, 1),    # W % 4 == 0, long tile rows
    ops.ConvShape(1, 24, 40, 62, 50, 3, 3, 1, 1, 1, 1),
    ops.ConvShape(1, 12, 16, 20, 20, 3, 3, 1, 1, 0, 1),    # pad 0 rows, pad 1 columns
    ops.ConvShape(2, 256, 13, 13, 384, 3, 3, 1, 1, 1, 1),  # a conv-set layer (long K: many stages)
]


def check(out, s):
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1)
    nm, rl2, hyb = orc.normalized_errors(ref, out)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
    assert hyb <= WINO_ELEM_TOL, (s, hyb)


@pytest.mark.parametrize("cn", WG)
def test_wg_config(dev, cn):
    ci = boda_hip.tune_cfg_names(1).index(cn)
    ran = 0
    try:
        for s in SHAPES:
            outs = {}
            for splits in (0, 1, 2, 5, 11, 15, 20, 21, 31):
                dev.tune_set(1, ci, splits)
                try:
                    out = run_conv(dev, s)
                except boda_hip.UnsupportedError:
                    break  # W % 4 != 0 for a 16-B strip form, or the strip does not fit
                ran += 1
                check(out, s)
                np.testing.assert_array_equal(run_conv(dev, s), out)
                if splits == 0:
                    np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
                outs[splits] = out
                if splits >= 20:  # the separate combine kernel sums the same slabs in the same order
                    np.testing.assert_array_equal(out, outs[splits - 20])
                if cn.startswith("wgl"):  # the lean transform makes the same V: bitwise the wgi route
                    dev.tune_set(1, boda_hip.tune_cfg_names(1).index("wgi" + cn[3:]), splits)
                    np.testing.assert_array_equal(run_conv(dev, s), out)
                    dev.tune_set(1, ci, splits)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 8, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", WG)
def test_wg_rejects_other_shapes(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        with pytest.raises(boda_hip.UnsupportedError):  # 5x5
            run_conv(dev, ops.ConvShape(1, 32, 28, 28, 16, 5, 5, 1, 1, 2, 2))
        with pytest.raises(boda_hip.UnsupportedError):  # stride 2
            run_conv(dev, ops.ConvShape(1, 16, 28, 28, 16, 3, 3, 2, 2, 1, 1))
        with pytest.raises(boda_hip.UnsupportedError):  # IC % 4 != 0
            run_conv(dev, ops.ConvShape(1, 3, 28, 28, 16, 3, 3, 1, 1, 1, 1))
        with pytest.raises(boda_hip.UnsupportedError):  # pad 2
            run_conv(dev, ops.ConvShape(1, 16, 28, 28, 16, 3, 3, 1, 1, 2, 2))
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [n for n in WG if n in ("wgp64x64", "wgp128x32v")])
def test_wg_residual_and_slab(dev, cn):
    s = ops.ConvShape(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1)
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        plain = run_conv(dev, s, relu=0)
        n = s.B * s.OC * s.OH * s.OW
        r = (np.random.default_rng(3).standard_normal(n) * 3).astype(np.float32)
        i, f, b = dev.alloc_floats(s.B * s.IC * s.H * s.W), dev.alloc_floats(s.OC * s.K), dev.alloc_floats(s.OC)
        dr, o = dev.alloc_floats(n), dev.alloc_floats(n)
        dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
        dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
        dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
        dr.upload(r)
        dev.conv_res(i, f, b, dr, o, s, 1)
        exp = (plain + r).astype(np.float32)
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


@pytest.mark.parametrize("cn", [n for n in WG if n in ("wgp64x64v", "wgi128x32")])
def test_wg_dword_aligned_pointers(dev, cn):
    """Input and output pointers one float past a 16-B boundary (a caller's sub-buffer): the strip
    DMA takes any dword alignment, and the 8-B paired output stores fall back to dword stores."""
    s = ops.ConvShape(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1)
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
