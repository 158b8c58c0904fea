"""Resident-bank 1x1 kernels (bh_k1s.hip, configs ks*, their pixels-on-N form kn*, the whole-bank kd* and the
store-wave kw* and the register-bank kr*) against the oracle.

Each ks / kn configuration serves unpadded stride-1 1x1 convs whose input channels are a whole
number of its trips (Q chunks of KC channels: ks<OCT>c<KC>q<Q>, kn<OCT>p<pixels per unit>c<KC>q<Q>;
a kn unit of 32 TN pixels needs OH*OW % TN == 0, TN = pixels / 32). It is forced with bh_tune_set
on such shapes: pixel units that run across image boundaries (13x13, 7x9, 6x6 images), quads
that straddle an image (OH*OW % 4 != 0: element stores), ragged output channels and several OC
tiles, fewer pixels than one unit, and every blocks-per-CU setting the tuner may pick -- checked
against the double-accumulated oracle with the tolerances of test_gpu_conv.py.
The kernel has no cross-wave sums, so a rerun must give the same bits, and the residual /
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

KS = [n for n in boda_hip.tune_cfg_names(1) if n.startswith(("ks", "kn", "kd", "kw", "kr"))]


def trip_of(name):
    if name.startswith("kd"):  # kd<OCT>c<KC>d<D>w<NW>: K a multiple of KC (and >= (D - 1) KC: min_k)
        return int(re.match(r"kd\d+c(\d+)", name).group(1))
    kc, q = map(int, re.match(r"k[snwr]\d+(?:p\d+)?(?:k\d+)?c(\d+)q(\d+)", name).groups())
    return kc * q


def min_k(name):
    m = re.match(r"kd\d+c(\d+)d(\d+)", name)
    return int(m.group(1)) * (int(m.group(2)) - 1) if m else 0


def tn_of(name):
    """Pixels per lane of a kn configuration (1 for ks)."""
    if name.startswith(("kd", "kw")):  # kd: 16-B input pieces of 4 pixels; kw: 16-B output stores of 4 pixels
        return 4
    m = re.match(r"kn\d+p(\d+)", name)
    return int(m.group(1)) // 32 if m else 1


def fits(name, ic, oc=None, ohw=None):
    """ks: the bank slice [IC][OCT] and the waves' [32][36] epilogue tiles fit the LDS; kn: the
    bank slice and the tile's biases (whole 64-float DMAs); kd: the whole bank [IC][OC rounded to
    the sub-tile], the biases and every wave's ring [D][KC][32], with OH*OW % 4 == 0."""
    oct_ = int(re.match(r"k[sdnwr](\d+)", name).group(1))
    if name.startswith("kr"):  # the bank slice in registers: K <= KMAX, no LDS
        return ic <= int(re.match(r"kr\d+k(\d+)", name).group(1))
    if name.startswith("kw"):  # the bank slice in whole 64-lane 16-B DMAs, biases, staging slots, counters
        nw, nsl = map(int, re.match(r"kw\d+c\d+q\d+w(\d+)s\d+l(\d+)", name).groups())
        lds = -(-(ic * oct_ // 4) // 64) * 256 + -(-oct_ // 64) * 64 + nw * nsl * oct_ * 32 + 2 * nw
        return lds * 4 <= 160 * 1024 and ohw % 4 == 0
    if name.startswith("kd"):
        kc, d, nw = map(int, re.match(r"kd\d+c(\d+)d(\d+)w(\d+)", name).groups())
        ocp = -(-oc // oct_) * oct_
        return (ic * ocp + -(-ocp // 64) * 64 + nw * d * kc * 32) * 4 <= 160 * 1024 and ohw % 4 == 0 and ic >= min_k(name)
    if name.startswith("kn"):
        return (ic * oct_ + -(-oct_ // 64) * 64) * 4 <= 160 * 1024
    nw = 8 if name.endswith("w8") else 4
    return (ic * oct_ + nw * 32 * 36) * 4 <= 160 * 1024


def k1(b, ic, h, w, oc):
    return ops.ConvShape(b, ic, h, w, oc, 1, 1, 1, 1, 0, 0)


SHAPES = [k1(2, 96, 54, 54, 96), k1(1, 64, 56, 56, 64), k1(2, 192, 28, 28, 96),  # the conv set's big-pixel shapes
          k1(2, 96, 14, 14, 96), k1(3, 192, 13, 13, 70), k1(1, 96, 28, 28, 130), k1(5, 192, 6, 6, 64),
          k1(2, 96, 7, 9, 40), k1(2, 64, 14, 14, 64), k1(1, 128, 27, 27, 256), k1(3, 256, 7, 7, 48),
          k1(1, 288, 5, 5, 33), k1(1, 64, 1, 1, 20), k1(4, 384, 13, 13, 100),
          k1(2, 192, 12, 12, 72), k1(3, 128, 10, 10, 100)]  # OH*OW % 4 == 0, ragged OC: kn's masked rows


def check(out, s):
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b, s, 1)
    nm, rl2, _ = orc.normalized_errors(ref, out)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)


@pytest.mark.parametrize("cn", KS)
def test_ks_config(dev, cn):
    ci = boda_hip.tune_cfg_names(1).index(cn)
    ran = 0
    try:
        for s in SHAPES:
            if s.IC % trip_of(cn):
                continue
            if not fits(cn, s.IC, s.OC, s.OH * s.OW) or (s.OH * s.OW) % tn_of(cn):
                dev.tune_set(1, ci, 0)
                with pytest.raises(boda_hip.UnsupportedError):
                    run_conv(dev, s)
                continue
            for splits in (0, 1, 2):
                dev.tune_set(1, ci, splits)
                out = run_conv(dev, s)
                ran += 1
                check(out, s)
                np.testing.assert_array_equal(run_conv(dev, s), out)
                if splits == 0:
                    np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 6, "config %s ran on too few shapes" % cn


@pytest.mark.parametrize("cn", KS)
def test_ks_rejects(dev, cn):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    t = trip_of(cn)
    try:
        for s in (ops.ConvShape(1, t, 13, 13, 16, 3, 3, 1, 1, 1, 1),  # not 1x1
                  ops.ConvShape(1, t, 13, 13, 16, 1, 1, 2, 2, 0, 0),  # stride 2
                  ops.ConvShape(1, t, 13, 13, 16, 1, 1, 1, 1, 1, 1),  # padded
                  k1(1, t + 16, 13, 13, 16)):                          # K not a whole number of trips
            with pytest.raises(boda_hip.UnsupportedError):
                run_conv(dev, s)
        if min_k(cn) > t:  # fewer input channels than the ring's prologue holds
            with pytest.raises(boda_hip.UnsupportedError):
                run_conv(dev, k1(1, t, 12, 12, 16))
        if tn_of(cn) > 1:  # a lane's pixels would straddle two images
            with pytest.raises(boda_hip.UnsupportedError):
                run_conv(dev, k1(2, t, 7, 7, 16))
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn,s", [(cn, s) for cn in ("ks96c32q3", "ks64c16q4", "kn96p32c8q4w8", "kn64p64c16q3w8",
                                                    "kn32p128c16q4w4", "kd96c16d6w4", "kd64c16d6w4", "kd32c32d5w4",
                                                    "kw32c16q3w8s2l2", "kw96c8q4w4s1l1", "kr32k192c16q3w4")
                                  for s in (k1(2, 192, 14, 14, 96), k1(3, 192, 13, 13, 70), k1(2, 192, 12, 12, 72))
                                  if (s.OH * s.OW) % tn_of(cn) == 0])
def test_ks_residual_and_slab(dev, cn, s):
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
