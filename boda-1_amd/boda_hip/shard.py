"""Multi-GPU plumbing for op sweeps.

Ops are independent, so N GPUs of one node split an op list with no data-path
collective: one process per GPU (launched by torch.distributed.run), each
binding its own device through the C-ABI. The only communication is the
control plane (barrier, max / sum of timings) over gloo on the host.

  lpt_partition  greedy longest-processing-time split of an op list by cost
                 (the same algorithm as boda_hip_ops_prof --shard=k/n)
  plan_units     the units a sharded sweep deals out: every op, with the SGEMMs too big
                 for one rank's share cut into column panels (independent sub-ops)
  Dist           rank / world from the torchrun environment, gloo barrier and
                 max / sum reductions of host floats
"""
import os


def lpt_partition(costs, n):
    """Greedy LPT: items by descending cost (stable), each to the least-loaded bin
    (lowest index on ties). Returns n sorted index lists."""
    bins = [[] for _ in range(n)]
    load = [0.0] * n
    for i in sorted(range(len(costs)), key=lambda i: -costs[i]):
        j = min(range(n), key=lambda j: load[j])
        bins[j].append(i)
        load[j] += costs[i]
    return [sorted(b) for b in bins]


def plan_units(shapes, costs, n, panel_align=128, max_frac=0.5):
    """Units of work for an n-way sharded sweep: (op index, shape, cost) triples.

    Ops are independent (src/rtc_prof.cc:232-360), so LPT over whole ops is enough unless one
    op outweighs a rank's share: sgemm-ops-full's 12288^3 alone is ~40 % of the list, which
    would cap 8-way strong scaling near 2.5x. An SGEMM c[M][N] = sum_k a[k][M] b[k][N] with
    cost > max_frac * total / n is cut into P column panels c[:, Nj] = a^T b[:, Nj] -- each an
    independent M x nj x K SGEMM (no exchange: a panel is its own output slab) -- of widths that
    are multiples of panel_align, P the least count that brings every panel under the bound.
    Other ops (convolutions: at most ~0.2 % of this list each) stay whole. At n == 1 nothing is
    cut. Returns units in op order (panels of an op consecutive)."""
    from .ops import SgemmShape
    total = float(sum(costs))
    bound = max_frac * total / n if n > 1 else float("inf")
    units = []
    for i, (s, c) in enumerate(zip(shapes, costs)):
        if not isinstance(s, SgemmShape) or c <= bound:
            units.append((i, s, c))
            continue
        P = int(-(-c // bound))
        cols = -(-s.N // panel_align)  # panel_align-wide column groups
        P = max(1, min(P, cols))
        base, extra = divmod(cols, P)
        n0 = 0
        for j in range(P):
            w = min((base + (1 if j < extra else 0)) * panel_align, s.N - n0)
            sub = SgemmShape(s.M, w, s.K)
            units.append((i, sub, c * w / s.N))
            n0 += w
        assert n0 == s.N
    return units


def imbalance(loads):
    """max / mean of per-rank loads (1.0 = perfectly balanced)."""
    m = sum(loads) / len(loads)
    return max(loads) / m if m > 0 else 1.0


class Dist:
    """torchrun environment + gloo control plane (no-op at world size 1)."""

    def __init__(self, backend="gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend, rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def _reduce(self, x, op):
        if not self.dist:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._reduce(x, self.dist.ReduceOp.MAX if self.dist else None)

    def sum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM if self.dist else None)

    def gather_obj(self, obj):
        """All ranks' objects, in rank order (rank 0 uses it to write merged results)."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()
            self.dist = None
