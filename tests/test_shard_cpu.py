"""Multi-GPU sweep plumbing on CPU: gloo world_size 2 (no GPU needed).

The op sweep shards with no data-path collective; what must be
right is the partition (disjoint, complete, balanced, identical in the Python
bench and the C++ ops-prof --shard) and the control plane (barrier, max/sum
reductions, gather) that bench.py uses across ranks.
"""
import os
import subprocess
import sys

import pytest

from boda_hip import ops, runner
from boda_hip.shard import lpt_partition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = os.path.join(ROOT, "tests", "golden", "ops")
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_ops_prof")


def sigs_costs():
    o, _ = ops.read_ops(os.path.join(OPS, "op_sigs_full.txt"))
    return [runner.roofline_secs(ops.shape_of(x)) for x in o]


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_lpt_partition_is_disjoint_complete_balanced(n):
    costs = sigs_costs()
    parts = lpt_partition(costs, n)
    flat = sorted(i for p in parts for i in p)
    assert flat == list(range(len(costs)))
    loads = [sum(costs[i] for i in p) for p in parts]
    # LPT bound: max load <= total/n + largest item
    assert max(loads) <= sum(costs) / n + max(costs) + 1e-15


WORKER = r"""
import os, sys, json
sys.path[:0] = [%(root)r, %(pkg)r]
from boda_hip.shard import Dist, lpt_partition
d = Dist()
costs = [float(c) for c in range(1, 38)]
mine = lpt_partition(costs, d.world)[d.rank]
d.barrier()
mx = d.max(sum(costs[i] for i in mine))
tot = d.sum(sum(costs[i] for i in mine))
allp = d.gather_obj(mine)
if d.rank == 0:
    print(json.dumps({"max": mx, "tot": tot, "parts": allp}))
d.close()
"""


def test_gloo_world_size_2_control_plane(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER % {"root": ROOT, "pkg": os.path.join(ROOT, "boda-1_amd")})
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", "--master-port=29517", str(script)],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    costs = [float(c) for c in range(1, 38)]
    parts = lpt_partition(costs, 2)
    assert res["parts"] == parts
    assert res["tot"] == sum(costs)
    assert res["max"] == max(sum(costs[i] for i in p) for p in parts)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_cpp_shard_matches_python(n):
    """boda_hip_ops_prof --shard=k/n runs exactly the ops Python's LPT gives shard k."""
    fn = os.path.join(OPS, "conv-ops-1-5-20-nin-alex-gn.txt")
    o, _ = ops.read_ops(fn)
    parts = lpt_partition([runner.roofline_secs(ops.shape_of(x)) for x in o], n)
    for k in range(n):
        r = subprocess.run([BIN, "--list-shard=%d/%d" % (k, n), "--ops-fn=" + fn], capture_output=True, text=True,
                           check=True)
        assert [int(x) for x in r.stdout.split()] == parts[k]


def bench_units(n):
    from boda_hip.shard import plan_units
    shapes = []
    for f in ("sgemm-ops-full.txt", "conv-ops-1-5-20-nin-alex-gn.txt", "op_sigs_full.txt"):
        o, _ = ops.read_ops(os.path.join(OPS, f))
        shapes += [ops.shape_of(x) for x in o]
    costs = [runner.roofline_secs(s) for s in shapes]
    return shapes, costs, plan_units(shapes, costs, n)


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_bench_units_cover_the_workload(n):
    """bench.py's sharded workload: column panels of the big SGEMMs tile each op's output
    exactly (same M, K; widths sum to N; flops add up), nothing else is cut, and the LPT
    deal of the units over n ranks is disjoint, complete and within 10 % of even."""
    from boda_hip.shard import imbalance
    shapes, costs, units = bench_units(n)
    assert sorted({u[0] for u in units}) == list(range(len(shapes)))
    for i, s in enumerate(shapes):
        mine = [u for u in units if u[0] == i]
        if len(mine) > 1:
            assert isinstance(s, ops.SgemmShape)
            assert all(u[1].M == s.M and u[1].K == s.K for u in mine)
            assert sum(u[1].N for u in mine) == s.N
        else:
            assert mine[0][1] == s
    assert abs(sum(u[1].flops() for u in units) - sum(s.flops() for s in shapes)) == 0
    if n == 1:
        assert len(units) == len(shapes)
    parts = lpt_partition([u[2] for u in units], n)
    assert sorted(i for p in parts for i in p) == list(range(len(units)))
    assert imbalance([sum(units[i][2] for i in p) for p in parts]) <= 1.1


BENCH_WORKER = r"""
import os, sys, json
sys.path[:0] = [%(root)r, %(pkg)r]
import bench
from boda_hip.shard import Dist
d = Dist()
shapes, tags = bench.load_sets(bench.DEFAULT_SETS)
units, mine, pred = bench.shard_units(shapes, tags, d.world, d.rank)
allm = d.gather_obj([(u[0], u[1].__class__.__name__, list(u[1].__dict__.values())) for u in mine])
if d.rank == 0:
    print(json.dumps({"n": len(units), "parts": allm, "pred": pred}))
d.close()
"""


def test_bench_rank_partitions_gloo_ws2(tmp_path):
    """bench.py at world size 2 (gloo, CPU): the two ranks' unit lists are disjoint and together
    are exactly the planned units."""
    import json
    script = tmp_path / "bw.py"
    script.write_text(BENCH_WORKER % {"root": ROOT, "pkg": os.path.join(ROOT, "boda-1_amd")})
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", "--master-port=29518", str(script)],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    a, b = [[tuple([x[0], x[1]] + x[2]) for x in p] for p in res["parts"]]
    assert a and b
    _, _, units = bench_units(2)
    planned = sorted(tuple([u[0], u[1].__class__.__name__] + list(u[1].__dict__.values())) for u in units)
    assert sorted(a + b) == planned
    assert len(a) + len(b) == res["n"] == len(units)
    assert res["pred"] <= 1.1
