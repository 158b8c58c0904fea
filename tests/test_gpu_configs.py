"""Every instantiated tile configuration, with and without split-K, against the oracle.

The tuning table (boda-1_amd/tuning/gfx950.tune) may route any op to any
configuration, so each one is checked on shapes that exercise ragged M/N/K
edges, both A loaders (K % 4 == 0 or not) and both B loaders (1x1 and im2col).
Tolerances as in test_gpu_conv.py.
"""
import re

import numpy as np
import pytest

import boda_hip
from boda_hip import ops
from oracle import oracle as orc
from test_gpu_conv import run_conv
from test_gpu_sgemm import kat_expect, run_sgemm

pytestmark = pytest.mark.gpu

CONV_SHAPES = [
    ops.ConvShape(2, 24, 11, 9, 70, 3, 3, 1, 1, 1, 1),   # im2col, K = 216 (% 4 == 0)
    ops.ConvShape(3, 5, 9, 13, 37, 3, 3, 2, 1, 1, 0),    # im2col, K = 45 (A scalar), stride 2
    ops.ConvShape(2, 132, 7, 5, 150, 1, 1, 1, 1, 0, 0),  # 1x1, K = 132
    ops.ConvShape(1, 17, 6, 6, 33, 1, 1, 1, 1, 0, 0),    # 1x1, K = 17 (A scalar)
    ops.ConvShape(2, 40, 8, 8, 20, 1, 1, 1, 1, 0, 0),    # 1x1, OH*OW % 4 == 0 (float4 output rows)
    ops.ConvShape(1, 8, 6, 6, 48, 3, 3, 1, 1, 1, 1),     # im2col, OH*OW % 4 == 0
    ops.ConvShape(1, 520, 4, 4, 40, 1, 1, 1, 1, 0, 0),   # 1x1, long K (register ring wraps)
    ops.ConvShape(2, 70, 9, 7, 40, 3, 3, 1, 1, 1, 1),    # im2col, IC >= BK (ring: two-tap loader), ragged
    ops.ConvShape(1, 64, 12, 11, 96, 5, 5, 2, 2, 2, 2),  # im2col 5x5 stride 2, IC = 64
    ops.ConvShape(2, 96, 13, 13, 100, 3, 3, 1, 1, 1, 1), # IC % BK == 0: one-tap K tiles (soffset loader), ragged M
    ops.ConvShape(2, 64, 9, 7, 70, 1, 1, 1, 1, 0, 0),    # 1x1, K % BK == 0 (soffset 1x1 loader), ragged N
    ops.ConvShape(1, 256, 5, 5, 130, 1, 1, 1, 1, 0, 0),  # 1x1, K = 256 in several K tiles / splits
]


# direct-conv configs (dc*) serve only their own kernel size / stride: tests/test_gpu_direct.py;
# gvp* only IC % 16 == 0: test_conv_gvp below; ks* (1x1): test_gpu_k1s.py; wg* (Winograd 3x3):
# test_gpu_wino.py; wx* (position-split Winograd 3x3 / 5x5): test_gpu_wgx.py
@pytest.mark.parametrize("ci", [i for i, n in enumerate(boda_hip.tune_cfg_names(1))
                                if not n.startswith(("dc", "dm", "gvp", "gvs", "gvo", "fcv", "ks", "kn", "kd", "kw", "kr", "wg", "wx"))],
                         ids=lambda i: boda_hip.tune_cfg_names(1)[i])
@pytest.mark.parametrize("splits", [1, 3, -3])
def test_conv_config(dev, ci, splits):
    dev.tune_set(1, ci, splits)
    try:
        for s in CONV_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            ref = orc.conv_ref(i, f, b, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            # a bank transformed up front (bh_conv_filts_pack) gives the same bits
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("ci", range(len(boda_hip.tune_cfg_names(0))),
                         ids=lambda i: boda_hip.tune_cfg_names(0)[i])
@pytest.mark.parametrize("splits", [1, 4, -4])
def test_sgemm_config(dev, ci, splits):
    dev.tune_set(0, ci, splits)
    try:
        for M, N, K in [(300, 260, 520), (96, 44, 301), (33, 17, 129)]:
            out = run_sgemm(dev, M, N, K, 600).reshape(M, N)
            np.testing.assert_array_equal(out, kat_expect(M, N, K))
            out = run_sgemm(dev, M, N, K, 5)
            a, b = orc.gen_sgemm(M, N, K, 5)
            nm, rl2, _ = orc.normalized_errors(orc.sgemm_ref(a, b, M, N, K), out)
            assert nm <= 1e-4 and rl2 <= 1e-5
    finally:
        dev.tune_set(0, -1, 0)


def test_split_k_repeatable(dev):
    """The in-kernel combine resets its tickets and sums slabs in a fixed order: repeated
    calls give bitwise-identical results, and equal the reduce-kernel combine bitwise."""
    s = CONV_SHAPES[0]
    outs = []
    for splits in (4, 4, 4, -4):
        dev.tune_set(1, 0, splits)
        outs.append(run_conv(dev, s))
    dev.tune_set(1, -1, 0)
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_tune_set_rejects_unknown_config(dev):
    with pytest.raises(boda_hip.UnsupportedError):
        dev.tune_set(1, 1000, 0)


# Stream-K configurations (srk*: persistent grid, iterations dealt equally to blocks) on
# shapes whose blocks finish whole tiles in place AND share cut tiles through slabs.
SRK_CONV_SHAPES = [
    ops.ConvShape(16, 64, 64, 64, 100, 1, 1, 1, 1, 0, 0),  # 1x1, K = 64: several whole tiles per block
    ops.ConvShape(2, 64, 30, 30, 96, 3, 3, 1, 1, 1, 1),    # two-tap loader, every tile cut
    ops.ConvShape(2, 3, 50, 50, 64, 7, 7, 2, 2, 3, 3),     # IC < BK stem conv, stride 2
    ops.ConvShape(2, 48, 20, 20, 96, 3, 3, 1, 1, 1, 1),    # BK 32: two-tap loader; BK 16: one-tap
    ops.ConvShape(4, 40, 20, 20, 70, 1, 1, 1, 1, 0, 0),    # 1x1, K % BK != 0: per-row loader
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith("srk")])
@pytest.mark.parametrize("bpc", [1, 2, 5, 6])
def test_conv_streamk(dev, cn, bpc):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), bpc)
    try:
        for s in SRK_CONV_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            ref = orc.conv_ref(i, f, b, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            # fixed-order slab combine: bitwise repeatable
            np.testing.assert_array_equal(run_conv(dev, s), out)
    finally:
        dev.tune_set(1, -1, 0)


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(0) if n.startswith("srk")])
@pytest.mark.parametrize("bpc", [1, 2, 6])
def test_sgemm_streamk(dev, cn, bpc):
    dev.tune_set(0, boda_hip.tune_cfg_names(0).index(cn), bpc)
    try:
        for M, N, K in [(2048, 1024, 96), (1000, 1000, 1000), (384, 260, 2048)]:
            out = run_sgemm(dev, M, N, K, 600).reshape(M, N)
            np.testing.assert_array_equal(out, kat_expect(M, N, K))
        out = run_sgemm(dev, 640, 384, 700, 5)
        a, b = orc.gen_sgemm(640, 384, 700, 5)
        nm, rl2, _ = orc.normalized_errors(orc.sgemm_ref(a, b, 640, 384, 700), out)
        assert nm <= 1e-4 and rl2 <= 1e-5
    finally:
        dev.tune_set(0, -1, 0)


# Filter-streaming configurations (gv*: few output columns, bank read in its reference layout)
GV_SHAPES = [
    ops.ConvShape(5, 64, 6, 6, 300, 6, 6, 1, 1, 0, 0),    # fc-as-conv: window = input (B_FC), 5 columns
    ops.ConvShape(3, 520, 1, 1, 130, 1, 1, 1, 1, 0, 0),   # InnerProduct on 1x1 input (B_FC), ragged M
    ops.ConvShape(1, 96, 6, 6, 70, 1, 1, 1, 1, 0, 0),     # 1x1, 36 columns (B_IM1X1)
    ops.ConvShape(1, 40, 6, 6, 100, 3, 3, 1, 1, 1, 1),    # 3x3 pad 1, 36 columns (B_IM2COL)
    ops.ConvShape(2, 12, 5, 5, 33, 3, 3, 2, 2, 0, 0),     # stride 2, 8 columns
    ops.ConvShape(2, 48, 14, 14, 70, 3, 3, 1, 1, 1, 1),   # 392 columns: a 2-D tile grid
    ops.ConvShape(1, 200, 7, 7, 40, 1, 1, 1, 1, 0, 0),    # 1x1, 49 columns, K % 16 != 0
    # im2col gathers: tabulated (B_IMTAB) when a K chunk fits the table and KYX <= 31
    ops.ConvShape(2, 16, 7, 7, 40, 5, 5, 1, 1, 2, 2),     # 5x5 pad 2: 25 taps
    ops.ConvShape(1, 256, 5, 5, 24, 3, 3, 1, 1, 1, 1),    # K 2304: past small tables unless split
    ops.ConvShape(1, 8, 9, 9, 20, 7, 7, 1, 1, 3, 3),      # 49 taps: direct (untabulated) gathers
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1)
                                if n.startswith("gv") and not n.startswith(("gvp", "gvs", "gvo"))])
@pytest.mark.parametrize("splits", [0, 1, 5])
def test_conv_gv(dev, cn, splits):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), splits)
    try:
        for s in GV_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            ref = orc.conv_ref(i, f, b, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)  # fixed-order combine
    finally:
        dev.tune_set(1, -1, 0)


# Register streaming over the packed bank (gvp* / gvs*: IC % 16 == 0, one-tap / 1x1 scalar-offset
# loaders; gvs: the ring of single-group buffers, whole trips + tail): ragged M / N, K chunks ending inside a batch, taps in the padding, stride 2,
# rows past OC4, several images per column tile
GVP_SHAPES = [
    ops.ConvShape(1, 160, 7, 7, 320, 3, 3, 1, 1, 1, 1),   # the small 3x3 ops (K 1440)
    ops.ConvShape(2, 48, 14, 14, 70, 3, 3, 1, 1, 1, 1),   # ragged M (70), 392 columns
    ops.ConvShape(5, 32, 7, 7, 100, 5, 5, 1, 1, 2, 2),    # 5x5 pad 2, 245 columns
    ops.ConvShape(2, 64, 12, 11, 37, 5, 5, 2, 2, 2, 2),   # stride 2, OC 37 (OC4 40)
    ops.ConvShape(5, 832, 7, 7, 48, 1, 1, 1, 1, 0, 0),    # 1x1, K 832
    ops.ConvShape(3, 96, 6, 6, 70, 1, 1, 1, 1, 0, 0),     # 1x1, ragged
    ops.ConvShape(1, 16, 9, 9, 20, 3, 3, 1, 1, 0, 0),     # K = 144: one group per tap
    ops.ConvShape(4, 256, 6, 6, 130, 6, 6, 1, 1, 0, 0),   # fc-as-conv through the tap loader
    ops.ConvShape(1, 512, 7, 7, 64, 3, 3, 1, 1, 1, 1),    # K 4608: many whole ring trips per wave
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith(("gvp", "gvs")) and "xw" not in n])
@pytest.mark.parametrize("splits", [0, 1, 3, 7])
def test_conv_gvp(dev, cn, splits):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), splits)
    try:
        for s in GVP_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            ref = orc.conv_ref(i, f, b, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)  # fixed-order combine
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)  # pre-packed bank
        # host-made random operands (no symmetry a transposed row / k map could hide behind)
        rng = np.random.default_rng(7)
        for s in (GVP_SHAPES[1], GVP_SHAPES[3], GVP_SHAPES[5]):
            hi = rng.standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
            hf = rng.standard_normal(s.OC * s.K).astype(np.float32)
            hb = rng.standard_normal(s.OC).astype(np.float32)
            out = run_conv(dev, s, host_inputs=(hi, hf, hb))
            ref = orc.conv_ref(hi, hf, hb, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
        with pytest.raises(boda_hip.UnsupportedError):  # IC % 16 != 0
            run_conv(dev, ops.ConvShape(1, 24, 7, 7, 32, 3, 3, 1, 1, 1, 1))
    finally:
        dev.tune_set(1, -1, 0)


# gvo*: 1x1 convs over the reference-layout bank (16-B A loads along k), IC % 16 == 0
GVO_SHAPES = [s for s in GVP_SHAPES if s.KY == 1 and s.KX == 1] + [
    ops.ConvShape(20, 528, 4, 4, 128, 1, 1, 1, 1, 0, 0),  # 320 columns over 20 images
    ops.ConvShape(1, 1024, 7, 7, 50, 1, 1, 1, 1, 0, 0),   # long K, ragged M
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith("gvo") and "xw" not in n])
@pytest.mark.parametrize("splits", [0, 1, 3, 7])
def test_conv_gvo(dev, cn, splits):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), splits)
    try:
        for s in GVO_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            ref = orc.conv_ref(i, f, b, s, 1)
            nm, rl2, _ = orc.normalized_errors(ref, out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)  # fixed-order combine
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)  # the pack is unused
        rng = np.random.default_rng(11)
        s = GVO_SHAPES[1]
        hi = rng.standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
        hf = rng.standard_normal(s.OC * s.K).astype(np.float32)
        hb = rng.standard_normal(s.OC).astype(np.float32)
        out = run_conv(dev, s, host_inputs=(hi, hf, hb))
        nm, rl2, _ = orc.normalized_errors(orc.conv_ref(hi, hf, hb, s, 1), out)
        assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
        for bad in (ops.ConvShape(1, 32, 7, 7, 32, 3, 3, 1, 1, 1, 1), ops.ConvShape(1, 24, 7, 7, 32, 1, 1, 1, 1, 0, 0)):
            with pytest.raises(boda_hip.UnsupportedError):  # not 1x1 / IC % 16 != 0
                run_conv(dev, bad)
    finally:
        dev.tune_set(1, -1, 0)


# gvo* on ipconv / FC ops (window = the whole unpadded input, OH = OW = 1, K % 16 == 0): the
# input rows are the columns (B_FC, one 16-B load per column tile and k group)
GVO_FC_SHAPES = [
    ops.ConvShape(4, 256, 6, 6, 130, 6, 6, 1, 1, 0, 0),   # fc6-like, K 9216, ragged M
    ops.ConvShape(20, 64, 1, 1, 100, 1, 1, 1, 1, 0, 0),   # 1x1 over a 1x1 input, 20 columns
    ops.ConvShape(3, 128, 4, 4, 70, 4, 4, 1, 1, 0, 0),    # K 2048
    ops.ConvShape(1, 1024, 1, 1, 1000, 1, 1, 1, 1, 0, 0), # one column
    ops.ConvShape(17, 48, 2, 2, 33, 2, 2, 1, 1, 0, 0),    # K 192, ragged N and M
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith("gvo") and "xw" not in n])
@pytest.mark.parametrize("splits", [0, 1, 4])
def test_conv_gvo_ipconv(dev, cn, splits):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), splits)
    try:
        for s in GVO_FC_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            nm, rl2, _ = orc.normalized_errors(orc.conv_ref(i, f, b, s, 1), out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)  # fixed-order combine
        rng = np.random.default_rng(13)
        for s in (GVO_FC_SHAPES[0], GVO_FC_SHAPES[4]):
            hi = rng.standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
            hf = rng.standard_normal(s.OC * s.K).astype(np.float32)
            hb = rng.standard_normal(s.OC).astype(np.float32)
            out = run_conv(dev, s, host_inputs=(hi, hf, hb))
            nm, rl2, _ = orc.normalized_errors(orc.conv_ref(hi, hf, hb, s, 1), out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
        with pytest.raises(boda_hip.UnsupportedError):  # ipconv with K % 16 != 0
            run_conv(dev, ops.ConvShape(2, 5, 2, 2, 8, 2, 2, 1, 1, 0, 0))
    finally:
        dev.tune_set(1, -1, 0)


# fcv*: batch-streaming ipconv (a wave per bank rows, lanes along k; batch <= the config's n<NB>)
FCV_SHAPES = [
    ops.ConvShape(1, 256, 6, 6, 130, 6, 6, 1, 1, 0, 0),   # fc6-like, K 9216, ragged M
    ops.ConvShape(1, 4096, 1, 1, 1000, 1, 1, 1, 1, 0, 0), # fc8-like
    ops.ConvShape(1, 12, 3, 3, 37, 3, 3, 1, 1, 0, 0),     # K 108: a partial 256-k chunk
    ops.ConvShape(2, 128, 4, 4, 70, 4, 4, 1, 1, 0, 0),    # K 2048, batch 2
    ops.ConvShape(4, 1000, 1, 1, 33, 1, 1, 1, 1, 0, 0),   # batch 4, K % 256 != 0
    ops.ConvShape(5, 64, 2, 2, 50, 2, 2, 1, 1, 0, 0),     # batch 5
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith("fcv")])
def test_conv_fcv(dev, cn):
    nb = int(re.search(r"n(\d+)$", cn).group(1))
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), 0)
    ran = 0
    try:
        for s in FCV_SHAPES:
            if s.B > nb:
                with pytest.raises(boda_hip.UnsupportedError):  # batch past the config's
                    run_conv(dev, s)
                continue
            ran += 1
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            nm, rl2, _ = orc.normalized_errors(orc.conv_ref(i, f, b, s, 1), out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)  # fixed summation order
            hi = np.random.default_rng(17).standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
            hf = np.random.default_rng(18).standard_normal(s.OC * s.K).astype(np.float32)
            hb = np.random.default_rng(19).standard_normal(s.OC).astype(np.float32)
            out = run_conv(dev, s, host_inputs=(hi, hf, hb))
            nm, rl2, _ = orc.normalized_errors(orc.conv_ref(hi, hf, hb, s, 1), out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
        for bad in (ops.ConvShape(1, 32, 7, 7, 32, 3, 3, 1, 1, 1, 1),   # not an ipconv
                    ops.ConvShape(1, 16, 4, 4, 8, 4, 4, 1, 1, 1, 1)):   # padded window
            with pytest.raises(boda_hip.UnsupportedError):
                run_conv(dev, bad)
    finally:
        dev.tune_set(1, -1, 0)
    assert ran >= 3


# interleaved column tiles (names *xw*: column i of MFMA tile c = pixel run position CX*i + c; one
# CX-wide load per k): 1x1 convs with OH*OW % CX == 0
GVX_SHAPES = [
    ops.ConvShape(2, 64, 14, 14, 96, 1, 1, 1, 1, 0, 0),
    ops.ConvShape(3, 96, 6, 6, 70, 1, 1, 1, 1, 0, 0),      # ragged M, 108 columns
    ops.ConvShape(20, 528, 4, 4, 128, 1, 1, 1, 1, 0, 0),
    ops.ConvShape(1, 512, 14, 14, 50, 1, 1, 1, 1, 0, 0),   # long K, 196 columns (ragged last tile)
]


@pytest.mark.parametrize("cn", [n for n in boda_hip.tune_cfg_names(1) if n.startswith("gv") and "xw" in n])
@pytest.mark.parametrize("splits", [0, 1, 3])
def test_conv_gv_interleaved(dev, cn, splits):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cn), splits)
    try:
        for s in GVX_SHAPES:
            out = run_conv(dev, s)
            i, f, b = orc.gen_conv(s, 5)
            nm, rl2, _ = orc.normalized_errors(orc.conv_ref(i, f, b, s, 1), out)
            assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
            np.testing.assert_array_equal(run_conv(dev, s), out)
            np.testing.assert_array_equal(run_conv(dev, s, packed=True), out)
        rng = np.random.default_rng(5)
        s = GVX_SHAPES[1]
        hi = rng.standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
        hf = rng.standard_normal(s.OC * s.K).astype(np.float32)
        hb = rng.standard_normal(s.OC).astype(np.float32)
        out = run_conv(dev, s, host_inputs=(hi, hf, hb))
        nm, rl2, _ = orc.normalized_errors(orc.conv_ref(hi, hf, hb, s, 1), out)
        assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
        for bad in (ops.ConvShape(5, 832, 7, 7, 48, 1, 1, 1, 1, 0, 0),   # OH*OW = 49
                    ops.ConvShape(1, 32, 8, 8, 32, 3, 3, 1, 1, 1, 1)):   # not 1x1
            with pytest.raises(boda_hip.UnsupportedError):
                run_conv(dev, bad)
    finally:
        dev.tune_set(1, -1, 0)
