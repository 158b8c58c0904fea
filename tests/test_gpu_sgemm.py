"""GPU parity of bh_sgemm_kmajor against the oracle and the reference's known-good digests.

Bars:
  * mode-600 known-answer test c[m][n] = 1000*m + n: bit-exact (integer-valued,
    one non-zero term per sum), at every size including BASELINE's full sizes;
  * mode-5 vs the reference digest (test/good_tr/sgemm-gen5): mrd_comp at 2e-4;
  * vs the double-accumulated oracle: max|d|/max(1,max|ref|) <= 1e-4 and
    rel-L2 <= 1e-5 (fp32 tolerance written here, F11).
"""
import numpy as np
import pytest

import boda_hip
from boda_hip import GEN_SGEMM_A, GEN_SGEMM_B
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

NORM_TOL, RL2_TOL = 1e-4, 1e-5


def run_sgemm(dev, M, N, K, mode):
    a, b, c = dev.alloc_floats(K * M), dev.alloc_floats(K * N), dev.alloc_floats(M * N)
    dev.gen_data(GEN_SGEMM_A, a, [K, M], mode)
    dev.gen_data(GEN_SGEMM_B, b, [K, N], mode)
    dev.sgemm(a, b, c, M, N, K)
    out = c.download()
    for x in (a, b, c):
        x.free()
    return out


def kat_expect(M, N, K):
    m = np.arange(M, dtype=np.int64)[:, None]
    n = np.arange(N, dtype=np.int64)[None, :]
    return np.where(n < K, 1000 * m + n, 0).astype(np.float32)


@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (128, 128, 128), (2048, 2048, 2048), (100, 36, 70),
                                   (1, 1, 1), (129, 257, 33), (4096, 4096, 4096), (37, 5, 3000)])
def test_kat_600_exact(dev, M, N, K):
    out = run_sgemm(dev, M, N, K, 600).reshape(M, N)
    np.testing.assert_array_equal(out, kat_expect(M, N, K))


@pytest.mark.slow
@pytest.mark.parametrize("S", [8192, 12288])
def test_kat_600_exact_full_size(dev, S):
    out = run_sgemm(dev, S, S, S, 600).reshape(S, S)
    np.testing.assert_array_equal(out, kat_expect(S, S, S))


def test_gen_data_matches_oracle(dev):
    K, M = 37, 129
    for mode in (2, 3, 4, 5, 600):
        buf = dev.alloc_floats(K * M)
        dev.gen_data(GEN_SGEMM_A, buf, [K, M], mode)
        ga = buf.download()
        dev.gen_data(GEN_SGEMM_B, buf, [K, M], mode)
        gb = buf.download()
        buf.free()
        oa, ob = orc.gen_sgemm(M, M, K, mode)
        np.testing.assert_array_equal(ga, oa)
        np.testing.assert_array_equal(gb, ob)


@pytest.mark.parametrize("suite,mode", [("sgemm-gen600", 600), ("sgemm-gen5", 5)])
def test_reference_digest(dev, golden, suite, mode):
    ent = golden(suite)[0]
    op = boda_hip.ops.parse_op(ent["op"])
    s = boda_hip.ops.sgemm_shape(op)
    kg = orc.Digest.from_golden(ent["kgs"][0])
    out = run_sgemm(dev, s.M, s.N, s.K, mode)
    d = orc.Digest.of(out, kg.dims, kg.seed)
    fails, worst = kg.compare(d, 2e-4)
    assert fails == 0, "worst rd/tol %.3f" % worst
    if mode == 600:  # the KAT digest is bit-exact in the reference too
        np.testing.assert_array_equal(d.samps, kg.samps)


@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (384, 384, 384), (1000, 1000, 1000), (77, 131, 517),
                                   (2048, 64, 8), (8, 2048, 4096)])
def test_vs_oracle_mode5(dev, M, N, K):
    out = run_sgemm(dev, M, N, K, 5)
    a, b = orc.gen_sgemm(M, N, K, 5)
    ref = orc.sgemm_ref(a, b, M, N, K)
    nm, rl2, _ = orc.normalized_errors(ref, out)
    assert nm <= NORM_TOL and rl2 <= RL2_TOL, (nm, rl2)


def test_asymmetric_operands(dev):
    """a != b (mode 5 data is symmetric, F10): distinct host-made operands catch a/b swaps."""
    M, N, K = 96, 160, 48
    rng = np.random.default_rng(1)
    a = rng.standard_normal(K * M).astype(np.float32)
    b = rng.standard_normal(K * N).astype(np.float32)
    da, db, dc = dev.alloc_floats(K * M), dev.alloc_floats(K * N), dev.alloc_floats(M * N)
    da.upload(a)
    db.upload(b)
    dev.sgemm(da, db, dc, M, N, K)
    out = dc.download()
    ref = (a.reshape(K, M).astype(np.float64).T @ b.reshape(K, N).astype(np.float64)).ravel()
    nm, rl2, _ = orc.normalized_errors(ref.astype(np.float32), out)
    assert nm <= NORM_TOL and rl2 <= RL2_TOL
