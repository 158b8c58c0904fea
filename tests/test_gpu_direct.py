"""Direct-conv stem kernels (bh_direct.hip, configs dc*) against the oracle.

Each dc configuration is instantiated for one kernel size and stride (its name: dc<k>s<s>...);
it is forced with bh_tune_set on stem-like shapes of that kernel -- the conv set's own stems
(GoogLeNet 7x7 s2 p3, AlexNet 11x11 s4), ragged channel counts, input channels 1..4, pixel
tiles that straddle output rows and images, asymmetric padding -- and checked against the
double-accumulated oracle (tolerances of test_gpu_conv.py). Bits must not
depend on whether the bank was packed up front, and the residual / channel-slab epilogues
must equal the plain call's bits (what the net executor relies on). Configurations ending in "p"
store the strip phase-split (column c at (c % S) * WPM / S + c / S) and read it through per-step
compile-time bases.
"""
import re

import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops
from oracle import oracle as orc
from test_gpu_conv import run_conv

pytestmark = pytest.mark.gpu

DC = [n for n in boda_hip.tune_cfg_names(1) if n.startswith("dc")]

SHAPES = {
    (7, 2): [ops.ConvShape(2, 3, 35, 35, 16, 7, 7, 2, 2, 3, 3),
             ops.ConvShape(1, 3, 224, 224, 64, 7, 7, 2, 2, 3, 3),
             ops.ConvShape(3, 3, 227, 227, 96, 7, 7, 2, 2, 0, 0),
             ops.ConvShape(2, 1, 60, 41, 70, 7, 7, 2, 2, 1, 3),
             ops.ConvShape(1, 4, 97, 100, 33, 7, 7, 2, 2, 2, 0),
             ops.ConvShape(2, 2, 40, 44, 20, 7, 7, 2, 2, 1, 1),    # W % 4 == 0, pad 1 (16-B strip)
             ops.ConvShape(2, 3, 128, 128, 40, 7, 7, 2, 2, 3, 3),   # W % 4 == 0, 2-row pixel tiles
             ops.ConvShape(2, 2, 90, 200, 40, 7, 7, 2, 2, 3, 3)],   # W % 4 == 0, IC <= 3: resident-weight 16-B strips
    (11, 4): [ops.ConvShape(2, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0),
              ops.ConvShape(1, 3, 224, 224, 96, 11, 11, 4, 4, 0, 0),
              ops.ConvShape(2, 2, 60, 71, 40, 11, 11, 4, 4, 2, 1),
              ops.ConvShape(1, 4, 120, 100, 100, 11, 11, 4, 4, 5, 5),
              ops.ConvShape(1, 4, 100, 224, 40, 11, 11, 4, 4, 1, 1),  # W % 4 == 0, pad 1 (16-B strip)
              ops.ConvShape(1, 3, 100, 516, 96, 11, 11, 4, 4, 0, 0),  # op_sigs' 516-wide stem rows
              ops.ConvShape(2, 2, 60, 300, 20, 11, 11, 4, 4, 2, 2),
              ops.ConvShape(2, 3, 60, 220, 40, 11, 11, 4, 4, 2, 2)],  # W % 4 == 0, IC 3: resident-weight 16-B strips
    (6, 2): [ops.ConvShape(1, 3, 100, 516, 40, 6, 6, 2, 2, 0, 0),    # op_sigs' 516-wide 6x6 s2 stem rows
             ops.ConvShape(2, 2, 64, 132, 20, 6, 6, 2, 2, 1, 1),     # 3-row pixel tiles, pad 1
             ops.ConvShape(1, 4, 40, 60, 33, 6, 6, 2, 2, 0, 2),
             ops.ConvShape(2, 3, 40, 508, 16, 6, 6, 2, 2, 1, 1)],    # 256-pixel tiles within two rows
    (11, 2): [ops.ConvShape(1, 3, 224, 224, 96, 11, 11, 2, 2, 0, 0),  # op_sigs' 11x11 s2 stem
              ops.ConvShape(1, 2, 60, 224, 24, 11, 11, 2, 2, 1, 1),
              ops.ConvShape(2, 3, 40, 100, 50, 11, 11, 2, 2, 3, 3)],
    (3, 1): [ops.ConvShape(1, 3, 224, 224, 64, 3, 3, 1, 1, 1, 1),
             ops.ConvShape(2, 3, 50, 210, 20, 3, 3, 1, 1, 1, 1),
             ops.ConvShape(1, 2, 40, 200, 70, 3, 3, 1, 1, 0, 2)],
}


def kernel_of(name):
    k, s = re.match(r"dc(\d+)s(\d+)", name).groups()
    return int(k), int(s)


def check(out, s):
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1)
    nm, rl2, _ = orc.normalized_errors(ref, out)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)


@pytest.mark.parametrize("cn", DC)
def test_direct_config(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    ran = 0
    try:
        for s in SHAPES[kernel_of(cn)]:
            try:
                out = run_conv(dev, s)
            except boda_hip.UnsupportedError:
                continue  # strip does not fit this instantiation (input too wide / too many rows)
            ran += 1
            check(out, s)
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
            np.testing.assert_array_equal(run_conv(dev, s), out)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 2, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", DC)
def test_direct_rejects_other_kernels(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    try:
        with pytest.raises(boda_hip.UnsupportedError):
            run_conv(dev, ops.ConvShape(1, 3, 30, 30, 16, 5, 5, 1, 1, 2, 2))
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [DC[0], [n for n in DC if n.startswith("dc11")][0]] + [n for n in DC if n == "dc11s4x32d2p"])
def test_direct_residual_and_slab(dev, cn):
    k, st = kernel_of(cn)
    s = SHAPES[(k, st)][1]  # a conv-set stem: fits every instantiation of its kernel
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
        # channel slab of a wider output, other channels untouched
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
