"""Multi-GPU plumbing for op sweeps.

Ops are independent, so N GPUs of one node split an op list with no data-path
collective: one process per GPU (launched by torch.distributed.run), each
binding its own device through the C-ABI. The only communication is the
control plane (barrier, max / sum of timings) over gloo on the host.

  lpt_partition  greedy longest-processing-time split of an op list by cost
                 (the same algorithm as boda_hip_ops_prof --shard=k/n)
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
