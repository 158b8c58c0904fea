"""Every instantiated tile configuration, with and without split-K, against the oracle.

The tuning table (boda-1_amd/tuning/gfx950.tune) may route any op to any
configuration, so each one is checked on shapes that exercise ragged M/N/K
edges, both A loaders (K % 4 == 0 or not) and both B loaders (1x1 and im2col).
Tolerances as in test_gpu_conv.py.
"""
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
]


@pytest.mark.parametrize("ci", range(len(boda_hip.tune_cfg_names(1))),
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
