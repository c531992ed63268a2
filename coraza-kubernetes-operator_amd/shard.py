"""Multi-GPU sharding helpers: one process per GPU, requests
sharded with no data-path collective; the only exchange is the per-step
all-gather of the fixed-size per-GPU tally plus the max-over-ranks wall time
bench.py reports.  Backend-agnostic: RCCL ("nccl") on the GPU box, gloo for
the world-size-2 CPU tests.

Tally vector per rank (int64): the 7 gi_tally counters, the GI_SCORE_BINS
score histogram and one match count per top-level rule
(gi_tally_detail_get) -- ~4 x (n_rules + 71) bytes, latency-bound.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

TALLY_KEYS = ("n_req", "n_interrupted", "n_matched_any", "n_error", "bytes_scanned", "matched_total", "n_pa_void")
SCORE_BINS = 64  # GI_SCORE_BINS


def shard_seed(base: int, rank: int) -> int:
    """Each rank generates and inspects its own disjoint synthetic batch."""
    return base + rank


def balanced_slices(sizes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) request slices, one per rank, with near-equal byte
    totals (a request set sharded by bytes, not by count, so the 4-64 KB / 1 MB
    bodies of C3 / C5 do not make one rank the straggler).  Every slice's byte
    total is within one request of total / world."""
    sizes = np.asarray(sizes, dtype=np.int64)
    n = len(sizes)
    csum = np.concatenate([[0], np.cumsum(sizes)])
    total = int(csum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(csum, target, side="left"))
        # the nearer of the two candidate boundaries, never before the previous cut
        if k > 0 and abs(csum[k - 1] - target) <= abs(csum[min(k, n)] - target):
            k -= 1
        cuts.append(max(cuts[-1], min(k, n)))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


class TallyGather:
    """all_gather_into_tensor of every rank's tally vector (int64)."""

    def __init__(self, dist, world: int, device, n_rules: int = 0):
        import torch
        self.dist = dist
        self.world = world
        self.n_rules = n_rules
        self.width = len(TALLY_KEYS) + SCORE_BINS + n_rules
        self.local = torch.zeros(self.width, dtype=torch.int64, device=device)
        self.gathered = torch.zeros(self.width * world, dtype=torch.int64, device=device)

    def push(self, tally: Dict[str, int], detail: Optional[Dict] = None) -> None:
        import torch
        vec = [int(tally[k]) for k in TALLY_KEYS]
        if detail is not None:
            assert len(detail["rule_hits"]) == self.n_rules
            vec += [int(x) for x in detail["score_hist"]] + [int(x) for x in detail["rule_hits"]]
        else:
            vec += [0] * (SCORE_BINS + self.n_rules)
        self.local.copy_(torch.tensor(vec, dtype=torch.int64))
        self.dist.all_gather_into_tensor(self.gathered, self.local)

    def _row(self, r) -> Dict:
        k0 = len(TALLY_KEYS)
        out = dict(zip(TALLY_KEYS, (int(x) for x in r[:k0])))
        out["score_hist"] = [int(x) for x in r[k0:k0 + SCORE_BINS]]
        out["rule_hits"] = [int(x) for x in r[k0 + SCORE_BINS:]]
        return out

    def per_rank(self) -> List[Dict]:
        rows = self.gathered.view(self.world, self.width).tolist()
        return [self._row(r) for r in rows]

    def total(self) -> Dict:
        return self._row(self.gathered.view(self.world, self.width).sum(0).tolist())


def max_over_ranks(dist, value: float, device) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
