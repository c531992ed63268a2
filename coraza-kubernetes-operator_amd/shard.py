"""Multi-GPU sharding helpers: one process per GPU, requests
sharded with no data-path collective; the only exchange is the per-step
all-gather of the fixed-size per-GPU tally (gi_tally) plus the max-over-ranks
wall time bench.py reports.  Backend-agnostic: RCCL ("nccl") on the GPU box,
gloo for the world-size-2 CPU tests.
"""
from __future__ import annotations

from typing import Dict

TALLY_KEYS = ("n_req", "n_interrupted", "n_matched_any", "n_error", "bytes_scanned", "matched_total", "n_pa_void")


def shard_seed(base: int, rank: int) -> int:
    """Each rank inspects its own disjoint synthetic batch."""
    return base + rank


class TallyGather:
    """all_gather_into_tensor of the 7-counter tally (int64) of every rank."""

    def __init__(self, dist, world: int, device):
        import torch
        self.dist = dist
        self.world = world
        self.local = torch.zeros(len(TALLY_KEYS), dtype=torch.int64, device=device)
        self.gathered = torch.zeros(len(TALLY_KEYS) * world, dtype=torch.int64, device=device)

    def push(self, tally: Dict[str, int]) -> None:
        import torch
        self.local.copy_(torch.tensor([int(tally[k]) for k in TALLY_KEYS], dtype=torch.int64))
        self.dist.all_gather_into_tensor(self.gathered, self.local)

    def per_rank(self):
        rows = self.gathered.view(self.world, len(TALLY_KEYS)).tolist()
        return [dict(zip(TALLY_KEYS, (int(x) for x in r))) for r in rows]

    def total(self) -> Dict[str, int]:
        tot = self.gathered.view(self.world, len(TALLY_KEYS)).sum(0).tolist()
        return dict(zip(TALLY_KEYS, (int(x) for x in tot)))


def max_over_ranks(dist, value: float, device) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
