"""Pin the CPU oracle to the reference's own known-good digests (CPU only).

The reference cannot be built or run here, so the oracle is
pinned by the digests it stores in test/good_tr/*/wisdom.wis (decoded into
tests/golden/*.json by tests/golden/make_golden.py). Checks:
  * gen_data + SGEMM mode-600 KAT digest: every sample bit-exact;
  * SGEMM mode 5, and every conv op of conv-gen5, conv-debug,
    ops-prof-conv-3x3-cudnn-boda and conv-full-gen5: the reference's mrd_comp at
    its default 2e-4 (src/rtc_prof.cc:161), except the one documented outlier
    (conv-full-gen5 op 178, fp32 cancellation in the stored digest).
"""
import numpy as np
import pytest

from boda_hip import ops
from oracle import oracle as orc

# conv-full-gen5 op 178 == ops-prof-conv-3x3-cudnn-boda op 37 (same op, same stored digest)
KNOWN_REF_DIGEST_OUTLIERS = {ops.ConvShape(5, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1)}


def test_det_hash_rand_values():
    # fmix32 of small integers, scaled to [-5, 5)
    vals = [orc.det_hash_rand(i) for i in range(1000)]
    assert all(-5.0 <= v < 5.0 for v in vals)
    assert orc.det_hash_rand(0) == -5.0  # fmix32(0) == 0


def test_digest_plan_matches_fixture_sample_count(golden):
    for suite in ["sgemm-gen600", "conv-debug", "conv-gen5"]:
        for ent in golden(suite):
            for kg in ent["kgs"]:
                orc.Digest.from_golden(kg)  # raises if the plan disagrees


def sgemm_digest(golden, suite, mode):
    ent = golden(suite)[0]
    s = ops.sgemm_shape(ops.parse_op(ent["op"]))
    kg = orc.Digest.from_golden(ent["kgs"][0])
    a, b = orc.gen_sgemm(s.M, s.N, s.K, mode)
    c = orc.sgemm_ref(a, b, s.M, s.N, s.K)
    return kg, orc.Digest.of(c, kg.dims, kg.seed)


def test_sgemm_gen600_bit_exact(golden):
    kg, d = sgemm_digest(golden, "sgemm-gen600", 600)
    assert d.min == kg.min and d.max == kg.max
    np.testing.assert_array_equal(d.samps, kg.samps)


def test_sgemm_gen5(golden):
    kg, d = sgemm_digest(golden, "sgemm-gen5", 5)
    fails, worst = kg.compare(d, 2e-4)
    assert fails == 0, worst


@pytest.mark.parametrize("suite", ["conv-gen5", "conv-debug", "ops-prof-conv-3x3-cudnn-boda", "conv-full-gen5"])
def test_conv_suites(golden, suite):
    bad = []
    for ix, ent in enumerate(golden(suite)):
        s = ops.conv_shape(ops.parse_op(ent["op"]))
        kg = orc.Digest.from_golden(ent["kgs"][0])
        inp, f, b = orc.gen_conv(s, 5)
        out = orc.conv_ref(inp, f, b, s, 1)
        fails, worst = kg.compare(orc.Digest.of(out, kg.dims, kg.seed), 2e-4)
        if fails and s not in KNOWN_REF_DIGEST_OUTLIERS:
            bad.append((ix, fails, worst))
        if s in KNOWN_REF_DIGEST_OUTLIERS:
            assert worst < 1.5, worst  # the documented ~1.2x miss, nothing worse
    assert not bad, bad


def test_fast_cpu_baseline_agrees_with_ref():
    s = ops.ConvShape(2, 16, 13, 11, 24, 3, 3, 2, 1, 1, 0)
    inp, f, b = orc.gen_conv(s, 5)
    ref = orc.conv_ref(inp, f, b, s, 1)
    fast = orc.conv_ref(inp, f, b, s, 1, fast=True)
    nm, rl2, _ = orc.normalized_errors(ref, fast)
    assert nm < 1e-5 and rl2 < 1e-6
    M, N, K = 67, 130, 300
    a, bb = orc.gen_sgemm(M, N, K, 5)
    nm, rl2, _ = orc.normalized_errors(orc.sgemm_ref(a, bb, M, N, K), orc.sgemm_ref(a, bb, M, N, K, fast=True))
    assert nm < 1e-5 and rl2 < 1e-6


def test_conv_out_size_rule():
    assert orc.conv_out_sz(227, 0, 11, 4) == 55
    assert orc.conv_out_sz(224, 3, 7, 2) == 112
    assert orc.conv_out_sz(2, 0, 5, 1) == 0
    for i, p, k, st in [(13, 1, 3, 1), (27, 2, 5, 1), (224, 0, 11, 4), (6, 0, 6, 1)]:
        assert orc.conv_out_sz(i, p, k, st) == ops.conv_out_sz(i, p, k, st)
