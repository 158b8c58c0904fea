"""The multi-GPU units on the GPU (BASELINE config C5).

bench.py at N > 1 deals the workload out as units (boda_hip.shard.plan_units): whole ops, and the
SGEMMs too big for one rank's share cut into column panels -- independent M x n_j x K SGEMMs, each
with its own contiguous operands (a K x M, b K x n_j, c M x n_j), which is what a rank times. Every
panel shape the planner makes at N = 2, 4, 8 runs here through its own route (table or heuristic)
against the mode-600 known answer c[m][n] = 1000 m + n (bit-exact, as test_gpu_sgemm.py), and the
ranks' unit lists are checked to cover the workload exactly once.
"""
import os

import numpy as np
import pytest

import boda_hip
from boda_hip import ops, runner
from boda_hip.shard import lpt_partition, plan_units
from test_gpu_sgemm import kat_expect, run_sgemm

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = os.path.join(ROOT, "tests", "golden", "ops")
LISTS = ["sgemm-ops-full.txt", "conv-ops-1-5-20-nin-alex-gn.txt", "op_sigs_full.txt"]


def workload():
    shapes = []
    for f in LISTS:
        o, _ = ops.read_ops(os.path.join(OPS, f))
        shapes += [ops.shape_of(x) for x in o]
    return shapes


def panels(n):
    shapes = workload()
    units = plan_units(shapes, [runner.roofline_secs(s) for s in shapes], n)
    return shapes, units, sorted({u[1] for u in units if u[1] != shapes[u[0]]}, key=lambda s: (s.M, s.N, s.K))


@pytest.mark.parametrize("n", [2, 4, 8])
def test_panel_units_kat(dev, n):
    shapes, units, pan = panels(n)
    assert pan, "the planner cuts no SGEMM at N=%d" % n
    for s in pan:
        assert isinstance(s, ops.SgemmShape)
        print(n, "panel", s, boda_hip.variant_name(0, [s.M, s.N, s.K]))
        out = run_sgemm(dev, s.M, s.N, s.K, 600).reshape(s.M, s.N)
        np.testing.assert_array_equal(out, kat_expect(s.M, s.N, s.K))
    # every op's panels tile its columns exactly; the ranks' units partition the list
    for i, s in enumerate(shapes):
        us = [u for u in units if u[0] == i]
        if isinstance(s, ops.SgemmShape):
            assert sum(u[1].N for u in us) == s.N and all((u[1].M, u[1].K) == (s.M, s.K) for u in us)
        else:
            assert [u[1] for u in us] == [s]
    parts = lpt_partition([u[2] for u in units], n)
    assert sorted(j for p in parts for j in p) == list(range(len(units)))
