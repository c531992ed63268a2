"""World-size-2 rehearsal of bench.py's multi-GPU path on CPU (gloo): the
per-rank tally all-gather (7 counters + score histogram + per-rule match
counts), its sum, the max-over-ranks timing and the byte-balanced request
split (coraza-kubernetes-operator_amd/shard.py).  No GPU needed."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


N_RULES = 5


def _detail(rank, step):
    return {"score_hist": [(rank + 1) * b * step for b in range(64)],
            "rule_hits": [(rank + 1) * 10 * (k + 1) + step for k in range(N_RULES)]}


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = shard.TallyGather(dist, world, "cpu", n_rules=N_RULES)
    for step in range(3):
        t = {k: (rank + 1) * (i + 1) * (step + 1) for i, k in enumerate(shard.TALLY_KEYS)}
        g.push(t, _detail(rank, step + 1))
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
    outs.sort(key=lambda o: o[0])
    for rank, tot, rows, m, seed in outs:
        # last step: rank r contributes (r+1)*(i+1)*3 to counter i
        for i, k in enumerate(shard.TALLY_KEYS):
            assert tot[k] == sum((r + 1) * (i + 1) * 3 for r in range(world))
            assert [row[k] for row in rows] == [(r + 1) * (i + 1) * 3 for r in range(world)]
        for r in range(world):
            assert rows[r]["score_hist"] == _detail(r, 3)["score_hist"]
            assert rows[r]["rule_hits"] == _detail(r, 3)["rule_hits"]
        assert tot["rule_hits"] == [sum(_detail(r, 3)["rule_hits"][k] for r in range(world)) for k in range(N_RULES)]
        assert tot["score_hist"] == [sum(_detail(r, 3)["score_hist"][b] for r in range(world)) for b in range(64)]
        assert m == pytest.approx(1.5 + world - 1)
        assert seed == 100 + rank


@pytest.mark.parametrize("world", [2, 3, 8])
def test_balanced_slices(world):
    import shard
    rng = np.random.default_rng(7)
    # C3-like: half GETs (~0.5 KB), half 4-64 KB log-uniform bodies, plus a few 1 MB outliers
    sizes = np.where(rng.random(5000) < 0.5, 500, np.exp(rng.uniform(np.log(4096), np.log(65536), 5000))).astype(int)
    sizes[rng.integers(0, 5000, 5)] = 1 << 20
    sl = shard.balanced_slices(sizes, world)
    assert sl[0][0] == 0 and sl[-1][1] == len(sizes)
    assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
    total, big = sizes.sum(), sizes.max()
    for lo, hi in sl:
        assert abs(sizes[lo:hi].sum() - total / world) <= big * 1.01


def test_take_and_request_bytes():
    import traffic
    b = traffic.TrafficGen(traffic.SEED).batch(40, post_frac=0.5)
    rb = b.request_bytes()
    assert int(rb.sum()) == b.raw_bytes()
    import shard
    parts = [b.take(lo, hi) for lo, hi in shard.balanced_slices(rb, 2)]
    assert sum(p.n_req for p in parts) == b.n_req
    assert sum(p.raw_bytes() for p in parts) == b.raw_bytes()
    assert parts[1].request(0) == b.request(parts[0].n_req)


def test_concat_roundtrip():
    import gpuinspect
    import traffic
    b = traffic.TrafficGen(traffic.SEED + 3).batch(30, post_frac=0.5)
    c = gpuinspect.concat([b.take(0, 7), b.take(7, 7), b.take(7, 30)])
    assert c.n_req == b.n_req
    assert [c.request(i) for i in range(c.n_req)] == [b.request(i) for i in range(b.n_req)]


def _rebalance_worker(rank, world, port, q):
    import hashlib

    import torch.distributed as dist

    import shard
    import traffic
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # this rank's chunk of the one request set (uneven on purpose: C3 bodies)
    chunk = traffic.TrafficGen(shard.shard_seed(traffic.SEED, shard.request_set_chunk(rank))).batch(
        40 + 30 * rank, post_frac=0.6)
    mine, rng, totals = shard.rebalance(dist, world, rank, chunk, "cpu")
    digs = [hashlib.sha1(repr(mine.request(i)).encode()).hexdigest() for i in range(mine.n_req)]
    q.put((rank, rng, totals, digs, int(mine.raw_bytes())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rebalance_one_request_set(world):
    """bench.py's multi-GPU split: ranks generate their chunks of one seeded
    request set and exchange requests so each holds a byte-balanced
    contiguous slice (gloo; the same code runs over RCCL on the GPU box)."""
    import hashlib

    import shard
    import traffic
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rebalance_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=180) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = [traffic.TrafficGen(shard.shard_seed(traffic.SEED, k)).batch(40 + 30 * k, post_frac=0.6) for k in range(world)]
    ref = [hashlib.sha1(repr(b.request(i)).encode()).hexdigest() for b in full for i in range(b.n_req)]
    sizes = np.concatenate([b.request_bytes() for b in full])
    assert [o[1] for o in outs] == shard.balanced_slices(sizes, world)
    assert sum((o[3] for o in outs), []) == ref  # the slices, in rank order, are the whole set
    for rank, (lo, hi), totals, digs, nbytes in outs:
        assert nbytes == totals[rank] == int(sizes[lo:hi].sum())
        assert abs(nbytes - sizes.sum() / world) <= sizes.max()


# ---------------------------------------------------------------- engine tallies
# tests/golden/tally_crs_pl1_world2.json: per-rank gi_tally / gi_tally_detail
# of one seeded CRS-PL1 request set cut into byte-balanced slices, recorded on
# an MI355X by tools/record_tally.py.  The CPU oracle pins the fixture
# (test_tally_fixture_matches_oracle); the gloo test all-gathers it the way
# bench.py --gpus 2 does and checks the node total.
TALLY_FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "tally_crs_pl1_world2.json")


def _fixture():
    import json
    return json.load(open(TALLY_FIXTURE))


def test_tally_fixture_matches_oracle():
    """The recorded engine tallies equal the oracle's, slice by slice."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import record_tally
    import shard
    from oracle import compare, coraza
    fx = _fixture()
    assert fx["seed"] == record_tally.SEED and fx["n_req"] > 0
    batch = record_tally.request_set(fx["n_req"])
    slices = shard.balanced_slices(batch.request_bytes(), fx["world"])
    cfg = coraza.parse_seclang(open(os.path.join(root, fx["ruleset"])).read())
    for (lo, hi), row in zip(slices, fx["ranks"]):
        assert row["slice"] == [lo, hi]
        part = batch.take(lo, hi)
        ov = compare.oracle_verdicts(cfg, part, tuple(fx["exports"]))
        assert not any(v.unsupported for v in ov.values())
        t = row["tally"]
        assert t["n_req"] == hi - lo
        assert t["bytes_scanned"] == int(part.request_bytes().sum())
        assert t["n_interrupted"] == sum(1 for v in ov.values() if v.rule_id or v.status)
        assert t["n_matched_any"] == sum(1 for v in ov.values() if v.matched)
        assert t["matched_total"] == sum(len(v.matched) for v in ov.values())
        assert t["n_error"] == 0 and t["n_pa_void"] == 0
        hits = {}
        for v in ov.values():
            for rid in v.matched:
                hits[rid] = hits.get(rid, 0) + 1
        assert {i: h for i, h in zip(row["rule_ids"], row["rule_hits"]) if h} == hits
        import gpuinspect
        hist = [0] * 64
        for v in ov.values():
            vals = []
            for e in fx["exports"]:
                a, ok = coraza.go_atoi(v.tx.get(e, b""))
                vals.append(a if ok else 0)
            hist[gpuinspect.score_hist_value(vals, fx["exports"])] += 1
        assert row["score_hist"] == hist
        assert sum(1 for x in hist if x) > 1  # the histogram carries information


def _fixture_worker(rank, world, port, q):
    import torch.distributed as dist

    import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    row = _fixture()["ranks"][rank]
    g = shard.TallyGather(dist, world, "cpu", n_rules=len(row["rule_ids"]))
    g.push(row["tally"], {"score_hist": row["score_hist"], "rule_hits": row["rule_hits"]})
    q.put((rank, g.total()))
    dist.barrier()
    dist.destroy_process_group()


def test_tally_gather_engine_fixture():
    """bench.py's N = 2 tally path over the recorded engine tallies."""
    fx = _fixture()
    world = fx["world"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fixture_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import shard
    rows = fx["ranks"]
    for _, tot in outs:
        for k in shard.TALLY_KEYS:
            assert tot[k] == sum(r["tally"][k] for r in rows)
        assert tot["n_req"] == fx["n_req"]
        assert tot["rule_hits"] == [sum(r["rule_hits"][k] for r in rows) for k in range(len(rows[0]["rule_ids"]))]
        assert tot["score_hist"] == [sum(r["score_hist"][b] for r in rows) for b in range(64)]
