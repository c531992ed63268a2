"""CRS-scale regex stress: 20 trie-assembled alternations
of 2-6 KB in the shape of CRS v4 942 / 932 / 941 (tools/gen_rxstress.py,
seeded), added to the PL1 stand-in as rulesets/crs_pl1_rxstress.conf.  Two of
them exceed the DFA state cap and run as NFA position tables.  The GPU test
compares verdicts with the oracle on C2-shaped traffic plus payloads built to
hit (and narrowly miss) every stress rule, in query args, cookies and an
urlencoded body."""
import os
import sys

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_rxstress  # noqa: E402

RS = os.path.join(ROOT, "rulesets", "crs_pl1_rxstress.conf")


def test_rxstress_file_is_generated():
    assert open(os.path.join(ROOT, "rulesets", "rxstress.conf")).read() == gen_rxstress.conf_text()
    sizes = [len(r[2]) for r in gen_rxstress.rules()]
    assert len(sizes) == 20 and min(sizes) >= 1800 and max(sizes) <= 6000


def test_rxstress_compiles_with_nfa_fallback():
    base = gpuinspect.Ruleset(open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read()).info
    info = gpuinspect.Ruleset(open(RS).read()).info
    assert info["n_rules"] == base["n_rules"] + 20
    assert info["n_nfas"] >= base["n_nfas"] + 2  # the wide-context rules are past the DFA state cap
    coraza.parse_seclang(open(RS).read())


def stress_batch(n_traffic=1200, seed=traffic.SEED + 11):
    txs = []
    for i, p in enumerate(gen_rxstress.payloads(n=120)):
        q = traffic._quote(p, i % 2 == 0)
        if i % 3 == 2:  # in an urlencoded body
            t = gpuinspect.Transaction(method=b"POST", uri=b"/submit")
            t.add_request_header("Host", "shop.example.com")
            t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
            t.write_request_body(b"name=x&comment=" + q)
        else:
            t = gpuinspect.Transaction(method=b"GET", uri=b"/search?q=" + q + b"&page=2")
            t.add_request_header("Host", "www.example.com")
            t.add_request_header("Cookie", "sid=" + p.decode(errors="replace").replace(";", "").replace(" ", ""))
        t.add_request_header("User-Agent", "Mozilla/5.0")
        txs.append(t)
    return gpuinspect.concat([gpuinspect.pack(txs), traffic.TrafficGen(seed).batch(n_traffic, attack_rate=0.3)])


@pytest.mark.gpu
def test_gpu_rxstress_parity():
    text = open(RS).read()
    batch = stress_batch()
    rs = gpuinspect.Ruleset(text)
    res = gpuinspect.Engine(rs, matched_cap=128).inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad[:5]
    fired = set()
    for v in orc.values():
        fired.update(m for m in v.matched if 942900 <= m < 942920)
    assert len(fired) >= 15, sorted(fired)  # the stress rules do fire (not vacuous)
