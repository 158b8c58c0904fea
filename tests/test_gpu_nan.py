"""A NaN in the input stays a NaN in the output of a conv without ReLU on every route, as in the
reference (src/cnn_codegen.cc:36,273: ReLU is max(0.0f, v); without ReLU the value is stored as is).
ADVICE r05: the resident-bank 1x1 (kn*) and resident-weight stem (dc*r*) epilogues took ReLU as one
v_max against a floor of -inf without ReLU, which turned a NaN into -inf; the floor is now a quiet NaN
(v_max_f32 returns the other operand)."""
import numpy as np
import pytest

import boda_hip
from boda_hip import ops
from oracle import oracle as orc
from test_gpu_conv import run_conv

pytestmark = pytest.mark.gpu

CASES = [("kn32p32c32q3w8", ops.ConvShape(2, 96, 14, 14, 96, 1, 1, 1, 1, 0, 0)),
         ("kn64p64c16q3w8", ops.ConvShape(2, 96, 12, 12, 72, 1, 1, 1, 1, 0, 0)),
         ("kw32c16q3w8s2l2", ops.ConvShape(2, 96, 14, 14, 96, 1, 1, 1, 1, 0, 0)),
         ("dc7s2r32d3v", ops.ConvShape(2, 3, 224, 224, 64, 7, 7, 2, 2, 3, 3)),
         ("dc11s4r32d2", ops.ConvShape(1, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0))]


@pytest.mark.parametrize("cn,s", CASES)
def test_nan_propagates_without_relu(dev, cn, s):
    names = boda_hip.tune_cfg_names(1)
    if cn not in names:
        pytest.skip("config %s not built" % cn)
    i, f, b = orc.gen_conv(s, 5)
    i = i.copy()
    # a NaN in image 0, channel 0 near the middle, and one in the last image's last channel
    hw = s.H * s.W
    i[(s.H // 2) * s.W + s.W // 2] = np.nan
    i[(s.B - 1) * s.IC * hw + (s.IC - 1) * hw + 5 * s.W + 7] = np.nan
    ref = orc.conv_ref(i, f, b, s, 0)
    dev.tune_set(1, names.index(cn), 0)
    try:
        got = run_conv(dev, s, relu=0, host_inputs=(i, f, b))
    finally:
        dev.tune_set(1, -1, 0)
    nan_ref = np.isnan(ref)
    assert nan_ref.any()
    np.testing.assert_array_equal(np.isnan(got), nan_ref)
    assert not np.isinf(got).any()
    ok = ~nan_ref
    nm, rl2, _ = orc.normalized_errors(ref[ok], got[ok])
    assert nm <= 1e-4 and rl2 <= 1e-5, (nm, rl2)
