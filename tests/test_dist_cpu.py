"""World-size-2 rehearsal of bench.py's multi-GPU path on CPU (gloo): the
per-rank tally all-gather, its sum, and the max-over-ranks timing
(coraza-kubernetes-operator_amd/shard.py).  No GPU needed."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = shard.TallyGather(dist, world, "cpu")
    for step in range(3):
        t = {k: (rank + 1) * (i + 1) * (step + 1) for i, k in enumerate(shard.TALLY_KEYS)}
        g.push(t)
    tot = g.total()
    rows = g.per_rank()
    m = shard.max_over_ranks(dist, 1.5 + rank, "cpu")
    q.put((rank, tot, rows, m, shard.shard_seed(100, rank)))
    dist.barrier()
    dist.destroy_process_group()


def test_tally_gather_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import shard
    outs.sort()
    for rank, tot, rows, m, seed in outs:
        # last step: rank r contributes (r+1)*(i+1)*3 to counter i
        for i, k in enumerate(shard.TALLY_KEYS):
            assert tot[k] == sum((r + 1) * (i + 1) * 3 for r in range(world))
            assert [row[k] for row in rows] == [(r + 1) * (i + 1) * 3 for r in range(world)]
        assert m == pytest.approx(1.5 + world - 1)
        assert seed == 100 + rank
