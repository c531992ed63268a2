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


def request_set_chunk(rank: int) -> int:
    """The request set a multi-GPU bench inspects is one seeded set: chunk k is
    the generator's batch for seed shard_seed(SEED, k), k = 0 .. world - 1,
    concatenated in order.  Each rank generates only its own chunk, then
    `rebalance` moves requests across chunk boundaries so every rank holds a
    byte-balanced contiguous slice of the whole set."""
    return rank


def _gather_i64(dist, x, device):
    import torch
    t = torch.as_tensor(np.asarray(x, dtype=np.int64), device=device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=device)
    world = dist.get_world_size()
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = int(max(int(v.item()) for v in ns))
    pad = torch.zeros(m, dtype=torch.int64, device=device)
    pad[:t.numel()] = t
    outs = [torch.zeros(m, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:int(k.item())].cpu().numpy() for o, k in zip(outs, ns)]


def _send_batch(dist, b, dst, device):
    import torch
    parts = [b.data.view(np.uint8), b.reqs.view(np.uint8), b.headers.view(np.uint8)]
    hdr = torch.tensor([len(p) for p in parts], dtype=torch.int64, device=device)
    dist.send(hdr, dst)
    for p in parts:
        if len(p):
            dist.send(torch.from_numpy(np.ascontiguousarray(p)).to(device), dst)


def _recv_batch(dist, src, device):
    import torch

    import gpuinspect
    hdr = torch.zeros(3, dtype=torch.int64, device=device)
    dist.recv(hdr, src)
    arrs = []
    for k in range(3):
        n = int(hdr[k].item())
        t = torch.zeros(n, dtype=torch.uint8, device=device)
        if n:
            dist.recv(t, src)
        arrs.append(t.cpu().numpy())
    return gpuinspect.PackedBatch(arrs[0], arrs[1].view(gpuinspect.REQUEST_DT), arrs[2].view(gpuinspect.HEADER_DT))


def rebalance(dist, world: int, rank: int, batch, device):
    """Byte-balanced split of one request set across ranks.

    `batch` is this rank's chunk of the set (request_set_chunk).  The ranks
    all-gather the raw byte size of every request, cut the concatenated set
    with balanced_slices, and send each request whose slice owner differs from
    its chunk owner to that rank (point-to-point, before any timing).  Returns
    (this rank's slice as a PackedBatch, (lo, hi) global range, per-rank byte
    totals)."""
    import gpuinspect
    sizes = _gather_i64(dist, batch.request_bytes(), device)
    counts = [len(x) for x in sizes]
    starts = np.concatenate([[0], np.cumsum(counts)])
    allsz = np.concatenate(sizes) if sizes else np.zeros(0, np.int64)
    sl = balanced_slices(allsz, world)
    pieces = {}
    # (owner s of chunk, receiver d of slice): every rank walks the pairs in one order
    for s in range(world):
        for d in range(world):
            lo = max(int(starts[s]), sl[d][0])
            hi = min(int(starts[s + 1]), sl[d][1])
            if hi <= lo:
                continue
            if s == d:
                if rank == s:
                    pieces[lo] = batch.take(lo - int(starts[s]), hi - int(starts[s]))
                continue
            if rank == s:
                _send_batch(dist, batch.take(lo - int(starts[s]), hi - int(starts[s])), d, device)
            elif rank == d:
                pieces[lo] = _recv_batch(dist, s, device)
    mine = gpuinspect.concat([pieces[k] for k in sorted(pieces)])
    totals = [int(allsz[a:b].sum()) for a, b in sl]
    return mine, sl[rank], totals


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
