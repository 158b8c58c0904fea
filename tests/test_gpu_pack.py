"""ABI 3 filter packs of chosen banks (include/boda_hip.h: bh_conv_filts_pack_banks,
bh_conv_route_banks, bh_conv2d_fwd_nchw_pkb) -- the role of Boda's xpose_filts made once per var
(test/rtc/xpose_filts.cucl, src/rtc_fwd.cc:306-326), sized to what the conv's route reads.

For 3x3 / 5x5 / 1x1 shapes under the table route and under forced routes of each bank kind (direct,
F(2x2,3x3), F(4x4,3x3), F(2x2,5x5)):
  * the route's bank mask names exactly the bank its kernel family reads;
  * a pack of just the route's banks gives the same output bits as the full ABI-2 pack, as the
    call without a pack, and -- its residual and channel-slab forms -- as _res / _slab;
  * a pack lacking the route's bank (k-major only) still gives the same bits (the call makes the
    bank itself);
  * sizes: k-major bank + the mask's banks, the full pack = every bank of the kernel size.
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import BANK_W23, BANK_W25, BANK_W43, BANKS_ALL, GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops

pytestmark = pytest.mark.gpu

C = ops.ConvShape
NAMES = boda_hip.tune_cfg_names(1)

CASES = [  # (shape, forced config or None for the table, expected bank)
    (C(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1), "wx43s8", BANK_W43),
    (C(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1), "wx23s6", BANK_W23),
    (C(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1), "wgp64x64v", BANK_W23),
    (C(2, 32, 28, 28, 96, 3, 3, 1, 1, 1, 1), "r64x64x32d4", 0),
    (C(2, 32, 28, 28, 96, 5, 5, 1, 1, 2, 2), "wx25s6", BANK_W25),
    (C(2, 32, 28, 28, 96, 5, 5, 1, 1, 2, 2), "dm5w32x64c4", 0),
    (C(20, 64, 56, 56, 192, 3, 3, 1, 1, 1, 1), None, None),   # table routes of the conv set
    (C(20, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2), None, None),
    (C(20, 256, 13, 13, 384, 3, 3, 1, 1, 1, 1), None, None),
    (C(20, 64, 56, 56, 64, 1, 1, 1, 1, 0, 0), None, 0),
]


def inputs(dev, s):
    i, f, b = dev.alloc_floats(s.B * s.IC * s.H * s.W), dev.alloc_floats(s.OC * s.K), dev.alloc_floats(s.OC)
    dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
    return i, f, b


def test_bank_sizes():
    s3, s5, s1 = C(1, 20, 9, 9, 40, 3, 3, 1, 1, 1, 1), C(1, 20, 9, 9, 40, 5, 5, 1, 1, 2, 2), C(1, 20, 9, 9, 40, 1, 1, 1, 1, 0, 0)
    km = lambda s: ((s.IC * s.KY * s.KX + 63) // 64 * 64) * ((s.OC + 3) // 4 * 4)
    w16, w36 = 20 * 64 * 16, 20 * 64 * 36  # [ceil4(IC)][ceil32(OC)][16 | 36]
    assert boda_hip.conv_filts_packed_floats(s3, 0) == km(s3)
    assert boda_hip.conv_filts_packed_floats(s3, BANK_W23) == km(s3) + w16
    assert boda_hip.conv_filts_packed_floats(s3, BANK_W43) == km(s3) + w36
    assert boda_hip.conv_filts_packed_floats(s3) == boda_hip.conv_filts_packed_floats(s3, BANKS_ALL) == km(s3) + w16 + w36
    assert boda_hip.conv_filts_packed_floats(s5) == km(s5) + w36
    assert boda_hip.conv_filts_packed_floats(s5, BANK_W23 | BANK_W43) == km(s5)  # not a 5x5's banks
    assert boda_hip.conv_filts_packed_floats(s1) == boda_hip.conv_filts_packed_floats(s1, BANKS_ALL) == km(s1)


@pytest.mark.parametrize("s,cn,bank", CASES, ids=["%s-%s" % ("x".join(map(str, c[0].as_dims())), c[1]) for c in CASES])
def test_route_pack(dev, s, cn, bank):
    if cn is not None:
        dev.tune_set(1, NAMES.index(cn), 0)
    try:
        rb = dev.route_banks(s)
        v = dev.variant(1, s.as_dims())
        if bank is not None:
            assert rb == bank, (v, rb)
        assert (rb != 0) == ("_wino_" in v), (v, rb)
        i, f, b = inputs(dev, s)
        n = s.B * s.OC * s.OH * s.OW
        outs = {}
        for tag, banks in (("full", BANKS_ALL), ("route", rb), ("kmajor", 0)):
            pk = dev.alloc_floats(boda_hip.conv_filts_packed_floats(s, banks))
            dev.conv_filts_pack(f, pk, s, banks)
            o = dev.alloc_floats(n)
            dev.conv_pkb(i, f, pk, banks, b, o, s)
            outs[tag] = o.download()
            if tag == "route":
                r = dev.alloc_floats(n)
                r.upload((np.random.default_rng(2).standard_normal(n) * 3).astype(np.float32))
                o2, o3 = dev.alloc_floats(n), dev.alloc_floats(n)
                dev.conv_pkb(i, f, pk, banks, b, o2, s, res=r)
                dev.conv_res(i, f, b, r, o3, s)  # no pack: the same route, its bank made in the call
                np.testing.assert_array_equal(o2.download(), o3.download())
                ctot, ofs = s.OC + 8, 5
                sl = dev.alloc_floats(s.B * ctot * s.OH * s.OW)
                sl.upload(np.full(s.B * ctot * s.OH * s.OW, -3.5, np.float32))
                dev.conv_pkb(i, f, pk, banks, b, sl, s, out_chans_total=ctot, out_chan_ofs=ofs)
                got = sl.download().reshape(s.B, ctot, s.OH, s.OW)
                np.testing.assert_array_equal(got[:, ofs:ofs + s.OC], outs["route"].reshape(s.B, s.OC, s.OH, s.OW))
                assert (got[:, :ofs] == -3.5).all() and (got[:, ofs + s.OC:] == -3.5).all()
                for x in (r, o2, o3, sl):
                    x.free()
            pk.free()
            o.free()
        o = dev.alloc_floats(n)
        dev.conv(i, f, b, o, s)
        outs["nopack"] = o.download()
        for x in (i, f, b, o):
            x.free()
        for tag in ("route", "kmajor", "nopack"):
            np.testing.assert_array_equal(outs[tag], outs["full"], err_msg=tag)
    finally:
        dev.tune_set(1, -1, 0)


def test_pkb_rejects_bad_slab(dev):
    s = C(1, 8, 9, 9, 16, 3, 3, 1, 1, 1, 1)
    i, f, b = inputs(dev, s)
    o = dev.alloc_floats(s.B * 20 * s.OH * s.OW)
    with pytest.raises(boda_hip.BodaHipError):  # slab past the tensor's channels
        dev.conv_pkb(i, f, None, 0, b, o, s, out_chans_total=20, out_chan_ofs=5)
    with pytest.raises(boda_hip.BodaHipError):  # residual with a slab
        dev.conv_pkb(i, f, None, 0, b, o, s, res=o, out_chans_total=20, out_chan_ofs=0)
    for x in (i, f, b, o):
        x.free()
