"""Multi-channel direct-conv kernels (bh_dcm.hip, configs dm*) against the oracle.

Each dm configuration serves one kernel size at stride 1 (its name: dm<k>w<pitch>...) and input
channel counts that are a multiple of its channel group (c<CI>). It is forced with bh_tune_set
on shapes of that kernel whose padded rows fit its strip pitch: pixel tiles that run across
image boundaries (13x13, 7x7, 6x6 images), ragged output channels, non-square and unpadded
inputs, and under every grid mode the tuner may pick (splits 0: stream-K at the occupancy's
blocks per CU, 1 / 2 blocks per CU, 5: whole tiles per block) -- checked against the
double-accumulated oracle with the tolerances of test_gpu_conv.py. A rerun
must give the same bits (the cut tiles are summed in a fixed block order), and the residual /
channel-slab epilogues must equal the plain call's bits.
"""
import re

import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops
from oracle import oracle as orc
from test_gpu_conv import run_conv

pytestmark = pytest.mark.gpu

DM = [n for n in boda_hip.tune_cfg_names(1) if n.startswith("dm")]

SHAPES = {
    3: [ops.ConvShape(2, 64, 13, 13, 96, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(1, 32, 14, 14, 130, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(3, 16, 7, 7, 70, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(5, 24, 6, 6, 40, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(2, 8, 11, 9, 33, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(1, 16, 15, 15, 32, 3, 3, 1, 1, 0, 0),
        ops.ConvShape(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(1, 16, 27, 30, 64, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(2, 16, 56, 56, 64, 3, 3, 1, 1, 1, 1),
        ops.ConvShape(1, 24, 40, 62, 50, 3, 3, 1, 1, 1, 1)],
    1: [ops.ConvShape(2, 64, 14, 14, 96, 1, 1, 1, 1, 0, 0),    # 16-B quads (OH*OW % 4 == 0)
        ops.ConvShape(3, 32, 13, 13, 70, 1, 1, 1, 1, 0, 0),    # dword (169 pixels per image)
        ops.ConvShape(1, 96, 28, 28, 130, 1, 1, 1, 1, 0, 0),
        ops.ConvShape(5, 160, 6, 6, 64, 1, 1, 1, 1, 0, 0),
        ops.ConvShape(2, 32, 7, 9, 40, 1, 1, 1, 1, 0, 0)],
    5: [ops.ConvShape(2, 32, 27, 27, 64, 5, 5, 1, 1, 2, 2),
        ops.ConvShape(1, 8, 28, 28, 40, 5, 5, 1, 1, 2, 2),
        ops.ConvShape(2, 12, 14, 14, 20, 5, 5, 1, 1, 2, 2),
        ops.ConvShape(3, 16, 14, 14, 48, 5, 5, 1, 1, 2, 2)],
}


def kernel_of(name):
    return int(re.match(r"dm(\d+)", name).group(1))


def check(out, s):
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1)
    nm, rl2, _ = orc.normalized_errors(ref, out)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)


@pytest.mark.parametrize("cn", DM)
def test_dm_config(dev, cn):
    ci = boda_hip.tune_cfg_names(1).index(cn)
    ran = 0
    try:
        for s in SHAPES[kernel_of(cn)]:
            for splits in (0, 1, 3, 6):
                dev.tune_set(1, ci, splits)
                try:
                    out = run_conv(dev, s)
                except boda_hip.UnsupportedError:
                    break  # strip does not fit this instantiation / channel group
                ran += 1
                check(out, s)
                np.testing.assert_array_equal(run_conv(dev, s), out)
                if splits == 0:
                    np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 3, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", DM)
def test_dm_rejects_other_kernels(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        with pytest.raises(boda_hip.UnsupportedError):
            run_conv(dev, ops.ConvShape(1, 32, 30, 30, 16, 7, 7, 1, 1, 3, 3))
        with pytest.raises(boda_hip.UnsupportedError):  # stride 2
            run_conv(dev, ops.ConvShape(1, 16, 13, 13, 16, kernel_of(cn), kernel_of(cn), 2, 2, 1, 1))
        k = kernel_of(cn)
        with pytest.raises(boda_hip.UnsupportedError):  # 3 input channels: not a multiple of any group
            run_conv(dev, ops.ConvShape(1, 3, 13, 13, 16, k, k, 1, 1, k // 2, k // 2))
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [n for n in DM if n in ("dm3w16x64c8", "dm5w32x64c4")])
def test_dm_residual_and_slab(dev, cn):
    s = SHAPES[kernel_of(cn)][0]
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
