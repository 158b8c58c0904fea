"""The same-node comparator (libboda_hip_vendor.so: rocBLAS sgemm, MIOpen conv+bias+ReLU) computes
the same op as the hand-written kernels on the same device buffers, so its per-op times in the
bench line (per_set.*.vendor_ms) are for identical work. fp32 tolerance: max|d| / max(1, max|ours|)
<= 1e-4 (different accumulation orders). Context only -- the vendor path is never the product."""
import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, GEN_SGEMM_A, GEN_SGEMM_B, ops, vendor

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def vd():
    v = vendor.Vendor(0)
    yield v
    v.close()


def _close(a, b):
    return np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))) <= TOL


@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (100, 36, 70), (1024, 512, 2048)])
def test_vendor_sgemm_matches_ours(dev, vd, M, N, K):
    a, b, c1, c2 = dev.alloc_floats(K * M), dev.alloc_floats(K * N), dev.alloc_floats(M * N), dev.alloc_floats(M * N)
    dev.gen_data(GEN_SGEMM_A, a, [K, M], 5)
    dev.gen_data(GEN_SGEMM_B, b, [K, N], 5)
    dev.sgemm(a, b, c1, M, N, K)
    dev.sync()
    vd.sgemm(a.ptr, b.ptr, c2.ptr, M, N, K)
    vd.sync()
    assert _close(c2.download(), c1.download())
    for x in (a, b, c1, c2):
        x.free()


@pytest.mark.parametrize("dims", [[5, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2], [1, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0],
                                  [20, 64, 56, 56, 64, 1, 1, 1, 1, 0, 0], [2, 17, 13, 11, 33, 3, 3, 2, 2, 1, 1]])
def test_vendor_conv_matches_ours(dev, vd, dims):
    s = ops.ConvShape(*dims)
    i, f, b = dev.alloc_floats(s.B * s.IC * s.H * s.W), dev.alloc_floats(s.OC * s.IC * s.KY * s.KX), \
        dev.alloc_floats(s.OC)
    o1, o2 = dev.alloc_floats(s.B * s.OC * s.OH * s.OW), dev.alloc_floats(s.B * s.OC * s.OH * s.OW)
    dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC, 1, 1, 1], 5)
    dev.conv(i, f, b, o1, s, relu=1)
    dev.sync()
    vd.conv(i.ptr, f.ptr, b.ptr, o2.ptr, s, relu=1)
    vd.sync()
    assert _close(o2.download(), o1.download())
    for x in (i, f, b, o1, o2):
        x.free()


def test_vendor_timing_reports(vd):
    t = vd.time(ops.SgemmShape(1024, 1024, 1024), 5)
    assert t["ms"] > 0 and t["lib"] == "rocblas_sgemm"
    t = vd.time(ops.ConvShape(5, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2), 5)
    assert t["ms"] > 0 and t["conv_only_ms"] > 0 and t["lib"].startswith("miopen:")
