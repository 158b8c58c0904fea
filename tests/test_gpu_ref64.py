"""The "ref64" configuration (bh_ref64.hip): conv and SGEMM summed in double and rounded once -- the
known-good tune of ops-prof sweeps (boda_hip_ops_prof --kg-tune-tag, src/rtc_prof.cc:276-321).

Forced with bh_tune_set, it must agree with the double-accumulated oracle element-wise to fp32
rounding (max min_sig_mag_rel_diff <= 1e-6, src/boda_base.cc:140-153), on ragged, strided, padded,
no-bias and residual / channel-slab shapes, and give the SGEMM known answer bit-exactly.
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import ops
from oracle import oracle as orc
from test_gpu_conv import run_conv
from test_gpu_sgemm import kat_expect, run_sgemm

pytestmark = pytest.mark.gpu
C = ops.ConvShape
SHAPES = [C(2, 24, 11, 9, 70, 3, 3, 1, 1, 1, 1), C(3, 5, 9, 13, 37, 3, 3, 2, 1, 1, 0), C(1, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0),
          C(5, 384, 13, 13, 256, 3, 3, 1, 1, 1, 1), C(2, 17, 6, 6, 33, 1, 1, 1, 1, 0, 0), C(2, 8, 5, 5, 16, 5, 5, 1, 1, 4, 4)]


@pytest.fixture
def ref64(dev):
    dev.tune_set(1, boda_hip.tune_cfg_names(1).index("ref64"), 0)
    dev.tune_set(0, boda_hip.tune_cfg_names(0).index("ref64"), 0)
    yield dev
    dev.tune_set(1, -1, 0)
    dev.tune_set(0, -1, 0)


@pytest.mark.parametrize("s", SHAPES, ids=lambda s: "x".join(map(str, s.as_dims())))
@pytest.mark.parametrize("bias", [True, False])
def test_ref64_conv(ref64, s, bias):
    assert ref64.variant(1, s.as_dims()) == "ref64_conv_double"
    out = run_conv(ref64, s, with_bias=bias)
    i, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(i, f, b if bias else None, s, 1)
    nm, rl2, hyb = orc.normalized_errors(ref, out)
    assert hyb <= 1e-6, (s, hyb)
    np.testing.assert_array_equal(run_conv(ref64, s, with_bias=bias, packed=True), out)


def test_ref64_residual_and_slab(ref64):
    s = SHAPES[0]
    plain = run_conv(ref64, s, relu=0)
    n = s.B * s.OC * s.OH * s.OW
    r = (np.random.default_rng(4).standard_normal(n) * 3).astype(np.float32)
    i, f, b = ref64.alloc_floats(s.B * s.IC * s.H * s.W), ref64.alloc_floats(s.OC * s.K), ref64.alloc_floats(s.OC)
    ref64.gen_data(boda_hip.GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    ref64.gen_data(boda_hip.GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    ref64.gen_data(boda_hip.GEN_CONV_BIASES, b, [s.OC], 5)
    dr, o = ref64.alloc_floats(n), ref64.alloc_floats(n)
    dr.upload(r)
    ref64.conv_res(i, f, b, dr, o, s, 1)
    exp = (plain + r).astype(np.float32)
    np.testing.assert_array_equal(o.download(), np.where(exp < 0, np.float32(0), exp))
    ctot, ofs = s.OC + 6, 3
    so = ref64.alloc_floats(s.B * ctot * s.OH * s.OW)
    so.upload(np.full(s.B * ctot * s.OH * s.OW, -1.5, np.float32))
    ref64.conv_slab(i, f, b, so, ctot, ofs, s)
    got = so.download().reshape(s.B, ctot, s.OH, s.OW)
    np.testing.assert_array_equal(got[:, ofs:ofs + s.OC], run_conv(ref64, s).reshape(s.B, s.OC, s.OH, s.OW))
    assert (got[:, :ofs] == -1.5).all() and (got[:, ofs + s.OC:] == -1.5).all()
    for x in (i, f, b, dr, o, so):
        x.free()


@pytest.mark.parametrize("mnk", [(300, 260, 520), (33, 17, 129), (1024, 1024, 1024)])
def test_ref64_sgemm(ref64, mnk):
    M, N, K = mnk
    assert ref64.variant(0, [M, N, K]) == "ref64_sgemm_double"
    np.testing.assert_array_equal(run_sgemm(ref64, M, N, K, 600).reshape(M, N), kat_expect(M, N, K))
    out = run_sgemm(ref64, M, N, K, 5)
    a, b = orc.gen_sgemm(M, N, K, 5)
    assert orc.normalized_errors(orc.sgemm_ref(a, b, M, N, K), out)[2] <= 1e-6
