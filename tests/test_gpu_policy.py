"""Output store policy (bh_tune_set_policy, tuning-table " wt=1"): write-through (sc1) output
stores give bit-identical results on every kernel family -- tile, ring, stream-K, register-
streaming (gv / gvp / gvs / gvo / fcv), direct stems (dc), multi-channel direct (dcm), resident-
bank 1x1 (ks) and the SGEMM ring -- and the variant name reports the policy. The direct kernels
(dc, dcm) keep write-back stores whatever the policy says (a policy branch at their deferred store
sites broke the counted waits), so their cases only check that the policy changes no bits."""
import numpy as np
import pytest

import boda_hip
from boda_hip import ops
from test_gpu_conv import run_conv
from test_gpu_sgemm import run_sgemm

pytestmark = pytest.mark.gpu

C = ops.ConvShape
CASES = [  # (shape, forced config or None for the table route)
    (C(2, 64, 14, 14, 96, 3, 3, 1, 1, 1, 1), "128x32x32"),
    (C(2, 64, 28, 28, 128, 3, 3, 1, 1, 1, 1), "r64x64x32d3"),
    (C(5, 384, 6, 6, 1024, 3, 3, 1, 1, 1, 1), None),         # gvs
    (C(1, 1024, 1, 1, 1000, 1, 1, 1, 1, 0, 0), None),        # fcv
    (C(1, 528, 14, 14, 128, 1, 1, 1, 1, 0, 0), None),        # gvo
    (C(5, 3, 224, 224, 96, 11, 11, 4, 4, 0, 0), None),       # dc stem (ignores the policy)
    (C(5, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2), None),         # dcm (ignores the policy)
    (C(2, 96, 54, 54, 96, 1, 1, 1, 1, 0, 0), "ks96c32q3"),   # k1s
    (C(3, 192, 13, 13, 70, 1, 1, 1, 1, 0, 0), "ks32c32q3"),  # k1s, quads across images
]


@pytest.mark.parametrize("s,cfg", CASES)
def test_write_through_same_bits(dev, s, cfg):
    if cfg:
        dev.tune_set(1, boda_hip.tune_cfg_names(1).index(cfg), 0)
    try:
        dev.tune_set_policy(1, 0)
        a = run_conv(dev, s)
        dev.tune_set_policy(1, 1)
        b = run_conv(dev, s)
    finally:
        dev.tune_set_policy(1, -1)
        dev.tune_set(1, -1, 0)
    np.testing.assert_array_equal(a, b)


def test_write_through_sgemm_and_name(dev):
    try:
        dev.tune_set_policy(0, 0)
        a = run_sgemm(dev, 2048, 2048, 2048, 5)
        dev.tune_set_policy(0, 1)
        b = run_sgemm(dev, 2048, 2048, 2048, 5)
    finally:
        dev.tune_set_policy(0, -1)
    np.testing.assert_array_equal(a, b)


def _table_entries():
    import os
    path = os.path.join(os.path.dirname(boda_hip.__file__), "..", "tuning", "gfx950.tune")
    for line in open(path):
        f = line.split()
        if len(f) >= 12 and f[0] == "conv":
            yield [int(x) for x in f[1:12]], "wt=1" in f


def test_variant_name_reports_policy():
    """A table entry with wt=1 names its variant with the _wt suffix; one without does not."""
    wt = [d for d, w in _table_entries() if w]
    wb = [d for d, w in _table_entries() if not w]
    assert wt and wb
    for d in wt[:8]:
        assert boda_hip.variant_name(1, d).endswith("_wt"), d
    for d in wb[:8]:
        assert not boda_hip.variant_name(1, d).endswith("_wt"), d
