"""Large rulesets (BASELINE.json configs[4], C5): generated @rx rules, a
phrase file split into phrase-group automata, multipart bodies -- and the
HBM-table scan launch (k_scan<false,false>) for automata beyond LDS.

CPU: generator determinism and compile plan.  GPU: a scaled C5 mix vs the
oracle, and the CRS mix with every job forced onto global tables
(GI_SCAN_HBM=1), bit-exact."""
import os

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def small_c5():
    return traffic.c5_ruleset(n_rx=300, n_phrases=12000)


def test_c5_generator_deterministic():
    a = traffic.c5_ruleset(n_rx=50, n_phrases=500)
    b = traffic.c5_ruleset(n_rx=50, n_phrases=500)
    assert a == b and a[0].count("@rx ") == 50
    x = traffic.c5_batch(2, body_bytes=20000, n_rx=50, n_phrases=500)
    y = traffic.c5_batch(2, body_bytes=20000, n_rx=50, n_phrases=500)
    assert bytes(x.data) == bytes(y.data) and x.raw_bytes() > 40000


def test_c5_small_compiles_with_phrase_groups():
    text, files = small_c5()
    rs = gpuinspect.Ruleset(text, data_files=files)
    # 300 exact @rx automata + phase-A unions + >= 3 phrase groups twice (operator + phase A)
    assert rs.info["n_rules"] == 303 and rs.info["n_dfas"] >= 306
    coraza.parse_seclang(text, files)


@pytest.mark.gpu
def test_gpu_c5_small_parity():
    text, files = small_c5()
    batch = traffic.c5_batch(8, body_bytes=65536, n_rx=300, n_phrases=12000, hit_rate=0.2)
    rs = gpuinspect.Ruleset(text, data_files=files)
    res = gpuinspect.Engine(rs).inspect(batch)
    cfg = coraza.parse_seclang(text, files)
    verdicts = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:3]
    assert any(len(v.matched) > 2 for v in verdicts.values())


@pytest.mark.gpu
def test_gpu_c5_2k_rules_256k_multipart_parity():
    # >= 2k generated rules over >= 256 KB multipart bodies, each request vs the oracle
    text, files = traffic.c5_ruleset(n_rx=2000, n_phrases=30000)
    batch = traffic.c5_batch(4, body_bytes=262144, n_rx=2000, n_phrases=30000, hit_rate=0.05)
    rs = gpuinspect.Ruleset(text, data_files=files)
    assert rs.info["n_rules"] >= 2000
    res = gpuinspect.Engine(rs).inspect(batch)
    cfg = coraza.parse_seclang(text, files)
    verdicts = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:3]
    assert all(len(v.matched) > 5 for v in verdicts.values())
    assert not any(int(v["flags"]) & 0x0F for v in res.verdicts)


def _c5_oracle_worker(args):
    text, files, blob, i, exports = args
    cfg = coraza.parse_seclang(text, files)
    b = gpuinspect.PackedBatch(*blob)
    return i, coraza.inspect(cfg, compare.oracle_request(b.request(i)), exports)


@pytest.mark.gpu
def test_gpu_c5_full_shape_parity():
    """BASELINE configs[4] at its configured shape: 10k generated @rx rules +
    a 100k-phrase @pmFromFile list over ~1 MB multipart bodies, each request
    against the oracle.  The oracle (~40 s per request) runs in one forked
    process per request while the engine compiles and inspects."""
    import multiprocessing as mp
    text, files = traffic.c5_ruleset()
    batch = traffic.c5_batch(2)
    assert batch.raw_bytes() > 2_000_000
    blob = (batch.data, batch.reqs, batch.headers)
    exports = ["anomaly_score"]
    with mp.get_context("fork").Pool(2) as pool:
        pending = pool.map_async(_c5_oracle_worker, [(text, files, blob, i, exports) for i in range(2)])
        rs = gpuinspect.Ruleset(text, tx_exports=exports, data_files=files)
        assert rs.info["n_rules"] == 10003
        res = gpuinspect.Engine(rs).inspect(batch)
        verdicts = dict(pending.get(timeout=110))
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:3]
    assert all(len(v.matched) > 50 and v.rule_id == 99100 for v in verdicts.values())
    assert not any(int(v["flags"]) & 0x0F for v in res.verdicts)


@pytest.mark.gpu
def test_gpu_scan_hbm_forced_parity():
    text = open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read()
    batch = traffic.TrafficGen(traffic.SEED + 3).batch(1500, post_frac=0.2)
    os.environ["GI_SCAN_HBM"] = "1"
    try:
        rs = gpuinspect.Ruleset(text)
        eng = gpuinspect.Engine(rs)
        res = eng.inspect(batch)
        names = [ln["name"] for ln in eng.stats()["launches"]]
    finally:
        del os.environ["GI_SCAN_HBM"]
    assert "k_scan_hbm" in names and "k_scan" not in names, names
    cfg = coraza.parse_seclang(text)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, batch, rs.exports))
    assert not bad, bad[:3]
