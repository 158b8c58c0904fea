"""GPU parity of bh_conv2d_fwd_nchw against the oracle and the reference's known-good digests.

Every op of every reference conv suite is run on the GPU with the reference's
gen_data mode 5 (seeds of test/rtc/gen_data_Convolution_*.cucl), ReLU fused
(ops-prof always fuses it, src/cnn_op.cc:335-337), and checked two ways:
  (i)  digest of `out` vs the reference's stored known-good digest with the
       reference's own mrd_comp at 2e-4 (src/rtc_prof.cc:161, boda_base.cc:284-310);
  (ii) full tensor vs the double-accumulated oracle:
       max|d|/max(1,max|ref|) <= 1e-4 and rel-L2 <= 1e-5;
  (iii) an op the table routes to a Winograd variant (*_wino_*) also meets Boda's own Winograd
       bar element-wise: max min_sig_mag_rel_diff(1, ref, out) <= 2e-3, the tolerance the
       reference's ops-prof gives cuDNN's 3x3 Winograd (src/rtc_prof.cc:314-319).
Known reference outlier: conv-full-gen5 op index 178 fails the
reference digest by ~1.2x even for the double oracle -- fp32 cancellation noise in
the stored GPU digest itself -- so for it (ii) is the bar and (i) is reported.
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, ops
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NORM_TOL, RL2_TOL = 1e-4, 1e-5
WINO_ELEM_TOL = 2e-3  # src/rtc_prof.cc:314-319
# Every other route, element by element, the a-priori bound of an fp32 sum of the op's terms in ANY
# order (Higham, accumulation error): |out - exact| <= gamma_n * (sum_k |in_k * w_k| + |bias|), gamma_n =
# n u / (1 - n u), u = 2^-24, with n = K + 64 roundings along a term's path (the products, the K-long
# sum, a split-K combine, the bias, the fp32 rounding of the oracle's double result). ReLU only
# shrinks differences. A flat min_sig_mag_rel_diff bar (1e-3, round 6's first form) cannot hold for
# every fp32 route: an output near 1 whose terms sum to |.| ~ 10^4 carries ~1e-3 of absolute error
# in any fp32 order (1x96x128^2->256 5x5 on r128x128x32d3: 1.56e-3, K = 2400) -- this bound scales
# with each element's own condition instead, and is tight enough to catch a dropped or doubled term
# of any but the smallest magnitude.
U32 = 2.0 ** -24


def fp32_sum_gamma(s):
    n = s.K + 64
    return n * U32 / (1 - n * U32)


def abs_terms(inp, filts, biases, s, idx=None):
    """sum_k |in_k * w_k| + |bias| per output (the magnitude the fp32 bound scales with)."""
    ai, af = np.abs(inp), np.abs(filts)
    ab = np.abs(biases) if biases is not None else None
    return orc.conv_ref(ai, af, ab, s, 0) if idx is None else orc.conv_ref_at(ai, af, ab, s, idx, 0)


def assert_elem_bound(ref, got, s, variant, mag):
    """Winograd routes: Boda's element bar (2e-3); every other route: the fp32 sum bound."""
    _, _, hyb = orc.normalized_errors(ref, got)
    if variant is not None and is_wino(variant):
        assert hyb <= WINO_ELEM_TOL, (s, variant, hyb)
        return hyb
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    lim = fp32_sum_gamma(s) * mag.astype(np.float64)
    r = d / np.maximum(lim, 1e-30)
    assert (d <= lim).all(), (s, variant, "worst |d| / bound %.3g at %d" % (r.max(), int(r.argmax())), hyb)
    return hyb
# conv-full-gen5 op 178 == ops-prof-conv-3x3-cudnn-boda op 37 (same op, same stored digest)
KNOWN_REF_DIGEST_OUTLIERS = {ops.ConvShape(5, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1)}


def run_conv(dev, s, mode=5, relu=1, with_bias=True, host_inputs=None, packed=False):
    i = dev.alloc_floats(s.B * s.IC * s.H * s.W)
    f = dev.alloc_floats(s.OC * s.K)
    b = dev.alloc_floats(s.OC)
    o = dev.alloc_floats(s.B * s.OC * s.OH * s.OW)
    if host_inputs is None:
        dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], mode)
        dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], mode)
        dev.gen_data(GEN_CONV_BIASES, b, [s.OC], mode)
    else:
        hi, hf, hb = host_inputs
        i.upload(hi)
        f.upload(hf)
        b.upload(hb)
    pk = None
    if packed:  # the filter-bank transform made up front (bh_conv_filts_pack), as ops-prof does
        pk = dev.alloc_floats(boda_hip.conv_filts_packed_floats(s))
        dev.conv_filts_pack(f, pk, s)
    dev.conv(i, f, b if with_bias else None, o, s, relu, packed=pk)
    out = o.download()
    for x in (i, f, b, o) + ((pk,) if pk is not None else ()):
        x.free()
    return out


def is_wino(variant):
    return "_wino_" in variant


def check_vs_oracle(out, s, mode=5, relu=1, with_bias=True, variant=None):
    """The normalized bars and the element bar of the route that ran (Winograd: 2e-3, others the fp32
    sum bound; variant None: the route of a call made with an override, checked as a direct route)."""
    inp, filts, biases = orc.gen_conv(s, mode)
    b = biases if with_bias else None
    ref = orc.conv_ref(inp, filts, b, s, relu)
    nm, rl2, hyb = orc.normalized_errors(ref, out)
    assert nm <= NORM_TOL and rl2 <= RL2_TOL, (s, nm, rl2, hyb)
    mag = None if variant is not None and is_wino(variant) else abs_terms(inp, filts, b, s)
    return assert_elem_bound(ref, out, s, variant, mag)


def test_gen_data_matches_oracle(dev):
    s = ops.ConvShape(2, 3, 5, 7, 6, 3, 2, 1, 1, 0, 0)
    for mode in (2, 3, 4, 5):
        i = dev.alloc_floats(s.B * s.IC * s.H * s.W)
        f = dev.alloc_floats(s.OC * s.K)
        b = dev.alloc_floats(s.OC)
        dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], mode)
        dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], mode)
        dev.gen_data(GEN_CONV_BIASES, b, [s.OC], mode)
        oi, of, ob = orc.gen_conv(s, mode)
        np.testing.assert_array_equal(i.download(), oi)
        np.testing.assert_array_equal(f.download(), of)
        np.testing.assert_array_equal(b.download(), ob)
        for x in (i, f, b):
            x.free()


SUITES = ["conv-gen5", "conv-debug", "ops-prof-conv-3x3-cudnn-boda", "conv-full-gen5"]


@pytest.mark.parametrize("suite", SUITES)
def test_reference_suite(dev, golden, suite):
    ents = golden(suite)
    digest_fail = []
    for ix, ent in enumerate(ents):
        s = ops.conv_shape(ops.parse_op(ent["op"]))
        out = run_conv(dev, s)
        check_vs_oracle(out, s, variant=dev.variant(1, s.as_dims()))
        kg = orc.Digest.from_golden(ent["kgs"][0])
        d = orc.Digest.of(out, kg.dims, kg.seed)
        fails, worst = kg.compare(d, 2e-4)
        if fails and s not in KNOWN_REF_DIGEST_OUTLIERS:
            digest_fail.append((ix, s, fails, worst))
    assert not digest_fail, digest_fail


EDGE = [
    ops.ConvShape(1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0),      # 1x1x1x1
    ops.ConvShape(3, 5, 9, 11, 7, 3, 3, 1, 1, 1, 1),     # ragged everything, K % 4 != 0
    ops.ConvShape(2, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0),  # AlexNet conv1 class, IC=3, s4
    ops.ConvShape(1, 3, 224, 224, 64, 7, 7, 2, 2, 3, 3),  # 7x7 s2 p3
    ops.ConvShape(2, 64, 15, 13, 33, 3, 3, 2, 2, 1, 1),   # stride 2, odd sizes
    ops.ConvShape(4, 256, 6, 6, 130, 6, 6, 1, 1, 0, 0),   # ipconv class: 1x1 output
    ops.ConvShape(1, 1024, 1, 1, 1000, 1, 1, 1, 1, 0, 0),  # fc as 1x1 conv on 1x1 input
    ops.ConvShape(5, 17, 13, 13, 300, 1, 1, 1, 1, 0, 0),  # 1x1 with odd channel count
    ops.ConvShape(2, 8, 5, 5, 16, 5, 5, 1, 1, 4, 4),      # pad > kernel/2 (output larger than input)
    ops.ConvShape(1, 2, 4, 4, 3, 4, 4, 3, 3, 0, 0),       # kernel == input (single output pixel)
    ops.ConvShape(1, 4, 10, 10, 8, 2, 3, 1, 2, 0, 1),     # asymmetric kernel / stride / pad
]


@pytest.mark.parametrize("s", EDGE, ids=lambda s: "x".join(map(str, s.as_dims())))
def test_edge_shapes(dev, s):
    out = run_conv(dev, s)
    check_vs_oracle(out, s)


def test_no_relu_no_bias(dev):
    s = ops.ConvShape(2, 16, 9, 9, 40, 3, 3, 1, 1, 1, 1)
    out = run_conv(dev, s, relu=0, with_bias=False)
    assert (out < 0).any()  # without ReLU negatives survive
    check_vs_oracle(out, s, relu=0, with_bias=False)


def test_asymmetric_filters(dev):
    """Host-made random data so filter/input roles cannot be confused by symmetric patterns."""
    s = ops.ConvShape(2, 6, 8, 10, 12, 3, 2, 1, 1, 1, 0)
    rng = np.random.default_rng(7)
    hi = rng.standard_normal(s.B * s.IC * s.H * s.W).astype(np.float32)
    hf = rng.standard_normal(s.OC * s.K).astype(np.float32)
    hb = rng.standard_normal(s.OC).astype(np.float32)
    out = run_conv(dev, s, relu=0, host_inputs=(hi, hf, hb))
    ref = orc.conv_ref(hi, hf, hb, s, 0)
    nm, rl2, _ = orc.normalized_errors(ref, out)
    assert nm <= NORM_TOL and rl2 <= RL2_TOL


def test_unsupported_is_reported(dev):
    s = ops.ConvShape(1, 1, 2, 2, 1, 5, 5, 1, 1, 0, 0)  # kernel larger than padded input
    with pytest.raises(boda_hip.UnsupportedError):
        run_conv(dev, s)


SLAB_SHAPES = [
    ops.ConvShape(20, 480, 14, 14, 64, 1, 1, 1, 1, 0, 0),  # 1x1, latency / ring kernels
    ops.ConvShape(20, 192, 28, 28, 128, 3, 3, 1, 1, 1, 1),  # 3x3 ring kernel
    ops.ConvShape(1, 832, 7, 7, 48, 1, 1, 1, 1, 0, 0),  # register-streaming kernel, OH*OW % 4 != 0
    ops.ConvShape(5, 160, 7, 7, 320, 3, 3, 1, 1, 1, 1),  # K-split combine
    ops.ConvShape(5, 32, 28, 28, 96, 5, 5, 1, 1, 2, 2),
    ops.ConvShape(2, 3, 35, 35, 16, 7, 7, 2, 2, 3, 3),  # stem (IC < BK)
]


@pytest.mark.parametrize("s", SLAB_SHAPES, ids=lambda s: "x".join(map(str, s.as_dims())))
def test_conv_writes_channel_slab(dev, s):
    """bh_conv2d_fwd_nchw_slab (a conv writing its channels of a Concat's output in place):
    the slab holds exactly the bits of the plain call, every other channel is untouched."""
    ref = run_conv(dev, s).reshape(s.B, s.OC, s.OH, s.OW)
    ofs, ctot = 16, s.OC + 40
    i = dev.alloc_floats(s.B * s.IC * s.H * s.W)
    f = dev.alloc_floats(s.OC * s.K)
    b = dev.alloc_floats(s.OC)
    o = dev.alloc_floats(s.B * ctot * s.OH * s.OW)
    dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
    o.upload(np.full(s.B * ctot * s.OH * s.OW, -7.25, np.float32))
    dev.conv_slab(i, f, b, o, ctot, ofs, s)
    got = o.download().reshape(s.B, ctot, s.OH, s.OW)
    with pytest.raises(boda_hip.BodaHipError):  # slab past the tensor's channels
        dev.conv_slab(i, f, b, o, ctot, ctot - s.OC + 1, s)
    for x in (i, f, b, o):
        x.free()
    np.testing.assert_array_equal(got[:, ofs:ofs + s.OC], ref)
    assert (got[:, :ofs] == -7.25).all() and (got[:, ofs + s.OC:] == -7.25).all()


@pytest.mark.parametrize("s", SLAB_SHAPES, ids=lambda s: "x".join(map(str, s.as_dims())))
@pytest.mark.parametrize("relu", [0, 1])
def test_conv_residual_epilogue(dev, s, relu):
    """bh_conv2d_fwd_nchw_res: out = relu?(conv + bias + res) bit-identical to the plain conv's
    stored output plus res, rounded once more (what a separate Eltwise SUM computes)."""
    plain = run_conv(dev, s, relu=0)
    n = s.B * s.OC * s.OH * s.OW
    r = (np.random.default_rng(7).standard_normal(n) * 3).astype(np.float32)
    i = dev.alloc_floats(s.B * s.IC * s.H * s.W)
    f = dev.alloc_floats(s.OC * s.K)
    b = dev.alloc_floats(s.OC)
    dr, o = dev.alloc_floats(n), dev.alloc_floats(n)
    dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
    dr.upload(r)
    dev.conv_res(i, f, b, dr, o, s, relu)
    got = o.download()
    for x in (i, f, b, dr, o):
        x.free()
    exp = (plain + r).astype(np.float32)
    if relu:
        exp = np.where(exp < 0, np.float32(0), exp)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("s", [ops.ConvShape(1, 128, 4, 4, 1024, 4, 4, 1, 1, 0, 0),     # fcv route (ipconv)
                               ops.ConvShape(1, 1024, 1, 1, 1000, 1, 1, 1, 1, 0, 0),    # fcv route (FC)
                               ops.ConvShape(1, 528, 14, 14, 128, 1, 1, 1, 1, 0, 0),    # gvo route (1x1)
                               ops.ConvShape(1, 528, 4, 4, 128, 1, 1, 1, 1, 0, 0)])     # gvo route
@pytest.mark.parametrize("which", ["in", "filts", "both"])
def test_dword_aligned_pointers_on_vector_routes(dev, s, which):
    """A dword-aligned but not 16-B-aligned input or filter pointer on a shape whose table route
    needs 16-B loads (fcv, gvo) computes through a fallback kernel instead of failing."""
    import boda_hip as bh
    ni, nf = s.B * s.IC * s.H * s.W, s.OC * s.K
    bi, bf = dev.alloc_floats(ni + 4), dev.alloc_floats(nf + 4)
    b, o = dev.alloc_floats(s.OC), dev.alloc_floats(s.B * s.OC * s.OH * s.OW)
    vi = bh.DevBuf(dev, bi.ptr + (4 if which in ("in", "both") else 0), ni * 4)
    vf = bh.DevBuf(dev, bf.ptr + (4 if which in ("filts", "both") else 0), nf * 4)
    dev.gen_data(GEN_CONV_IN, vi, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, vf, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC], 5)
    dev.conv(vi, vf, b, o, s, 1)
    check_vs_oracle(o.download(), s)
    for x in (bi, bf, b, o):
        x.free()
