"""hipGraph capture/replay of an op sweep gives bitwise the eager results.

Covers the launch-batching C-ABI (bh_capture_begin/end, bh_graph_launch) and that
split-K tickets reset correctly across back-to-back replays of one graph.
"""
import numpy as np
import pytest

from boda_hip import ops, runner

pytestmark = pytest.mark.gpu

SHAPES = [ops.ConvShape(1, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1),   # split-K (small grid)
          ops.ConvShape(20, 64, 28, 28, 96, 3, 3, 1, 1, 1, 1),
          ops.ConvShape(5, 1024, 1, 1, 1000, 1, 1, 1, 1, 0, 0),
          ops.SgemmShape(768, 768, 768),
          ops.SgemmShape(100, 260, 1000)]


def test_graph_replay_matches_eager(dev):
    wl = runner.Workload(dev, SHAPES)
    wl.step()
    dev.sync()
    eager = [wl.output(i) for i in range(len(SHAPES))]
    for v in wl.ops:
        v.bufs[-1].zero()
    g = wl.capture_step(stamp_base=0)
    for _ in range(3):
        dev.graph_launch(g)
    dev.sync()
    for i in range(len(SHAPES)):
        np.testing.assert_array_equal(wl.output(i), eager[i])
    ts = dev.stamps_read(0, len(SHAPES) + 1)
    assert all(b > a for a, b in zip(ts, ts[1:]))  # stamps advance between ops
    dev.graph_destroy(g)
    wl.free()


def test_time_next_call_covers_split_k_reduce(dev):
    """bh_time_next_call's events sit on the call's own first and last dispatch: positive,
    and not longer than a host-side event pair around the same call."""
    s = ops.ConvShape(1, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1)
    wl = runner.Workload(dev, [s])
    dev.tune_set(1, 0, -8)  # 8 splits combined by the separate reduce kernel: two dispatches
    try:
        wl.launch(0)
        t_kernel, t_pair = [], []
        for _ in range(5):
            b, e = dev.time_next_call()
            wl.launch(0)
            dev.sync()
            t_kernel.append(dev.elapsed_ms(b, e))
            b2 = dev.event()
            wl.launch(0)
            e2 = dev.event()
            dev.sync()
            t_pair.append(dev.elapsed_ms(b2, e2))
        dev.events_reset()
        assert min(t_kernel) > 0
        assert sorted(t_kernel)[2] <= sorted(t_pair)[2] * 1.05
    finally:
        dev.tune_set(1, -1, 0)
        wl.free()
