"""GPU parity on the exact shapes the tuning table routes (VERDICT r01 "parity holes").

boda-1_amd/tuning/gfx950.tune sends each exact shape to a specific kernel configuration x
K-split count x combine mode; the configuration tests (test_gpu_configs.py) prove every
configuration on small ragged shapes, the reference-digest suites (test_gpu_conv.py) the 204
conv-set ops. Here every OTHER shape the bench, the C5 op_sigs sweep and the C4 nets route is
run through its tuned route (packed bank, as ops-prof and bench.py call it):
  * SGEMM: every size of test/sgemm-ops-{tiny,small,full}.txt with the mode-600 known-answer
    data, c[m][n] = 1000 m + n -- bit-exact (mode-5 data is symmetric);
  * conv: every Convolution of op_sigs_full.txt and of the five nets at batch 1 / 5 / 20
    (tools/net_ops.py lists) not already in the conv set, against the double-accumulated
    oracle: the full tensor (tolerances of test_gpu_conv.py) up to 20 GFLOP,
    16384 sampled outputs of each larger op (oracle.conv_ref_at); an op routed to a Winograd
    variant element-wise within 2e-3 (min_sig_mag_rel_diff, src/rtc_prof.cc:314-319), every other route
    within the a-priori fp32 sum bound of each element (test_gpu_conv.assert_elem_bound).
Reference anchor for the net-level comparison: src/test_compute.cc:216-276.
"""
import os

import numpy as np
import pytest

from boda_hip import ops
from oracle import oracle as orc
from test_gpu_conv import abs_terms, assert_elem_bound, is_wino, run_conv
from test_gpu_sgemm import kat_expect, run_sgemm

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = os.path.join(ROOT, "tests", "golden", "ops")
TUNING = os.path.join(ROOT, "boda-1_amd", "tuning")


def shapes_of(path):
    o, _ = ops.read_ops(path)
    return [ops.shape_of(x) for x in o]


SGEMM = sorted({(s.M, s.N, s.K) for f in ("sgemm-ops-tiny.txt", "sgemm-ops-small.txt", "sgemm-ops-full.txt")
                for s in shapes_of(os.path.join(OPS, f))})

_base = set(shapes_of(os.path.join(OPS, "conv-ops-1-5-20-nin-alex-gn.txt")))
CONV = []
for _p in [os.path.join(OPS, "op_sigs_full.txt")] + [os.path.join(TUNING, "net-ops-b%d.txt" % b) for b in (20, 5, 1)]:
    for _s in shapes_of(_p):
        if isinstance(_s, ops.ConvShape) and _s not in _base and _s not in CONV:
            CONV.append(_s)


def test_table_routes_are_the_ones_run(dev):
    """Every table line's op runs its table configuration in this process (the table loaded, nothing
    overriding it), so the route tests here and in test_gpu_conv.py check what the bench runs."""
    wrong = []
    for line in open(os.path.join(TUNING, "gfx950.tune")):
        if line.startswith("#") or " cfg=" not in line:
            continue
        key, rest = line.split(" cfg=", 1)
        op, dims = key.split()[0], [int(x) for x in key.split()[1:]]
        cfg = rest.split()[0]
        v = dev.variant(0 if op == "sgemm" else 1, dims)
        if cfg not in v:
            wrong.append((key, cfg, v))
    assert not wrong, wrong[:10]


@pytest.mark.parametrize("mnk", SGEMM, ids=lambda t: "x".join(map(str, t)))
def test_sgemm_tuned_route_kat(dev, mnk):
    M, N, K = mnk
    out = run_sgemm(dev, M, N, K, 600).reshape(M, N)
    np.testing.assert_array_equal(out, kat_expect(M, N, K))


FULL_MAX_FLOPS = 2e10


@pytest.mark.parametrize("s", CONV, ids=lambda s: "x".join(map(str, s.as_dims())))
def test_conv_tuned_route(dev, s):
    out = run_conv(dev, s, packed=True)
    i, f, b = orc.gen_conv(s, 5)
    v = dev.variant(1, s.as_dims())
    idx = None
    if s.flops() <= FULL_MAX_FLOPS:
        ref = orc.conv_ref(i, f, b, s, 1)
        got = out
    else:
        idx = np.random.default_rng(11).choice(out.size, 16384, replace=False).astype(np.uint64)
        ref = orc.conv_ref_at(i, f, b, s, idx, 1)
        got = out[idx.astype(np.int64)]
    nm, rl2, hyb = orc.normalized_errors(ref, got)
    assert nm <= 1e-4 and rl2 <= 1e-5, (s, nm, rl2)
    # Winograd 2e-3 (src/rtc_prof.cc:314-319), every other route the fp32 sum bound per element
    assert_elem_bound(ref, got, s, v, None if is_wino(v) else abs_terms(i, f, b, s, idx))
