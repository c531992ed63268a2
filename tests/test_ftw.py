"""Offline go-ftw replay (coraza-kubernetes-operator_amd/ftw.py).

The CRS v4.23.0 regression YAMLs are a download (reference Makefile:195-206),
so tests/ftw/ holds an authored corpus in go-ftw's v2 format for the
CRS-shaped rules, run against rulesets/crs_ftw.conf (the X-CRS-Test
configuration, generate_coreruleset_configmaps.py:113-141: blocking
paranoia 4, DetectionOnly).  CPU: the loader, the reference's own override
list (ftw/ftw.yml:4-72, read when /root/reference is present) and the
corpus's expectations against the oracle.  GPU: the replay through
gi_inspect_batch, every non-ignored test passing, verdicts bit-exact with
the oracle.
"""
import os

import pytest

import ftw
import gpuinspect
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CORPUS = os.path.join(ROOT, "tests", "ftw")
RULES = os.path.join(ROOT, "rulesets", "crs_ftw.conf")
REF_FTW = "/root/reference/ftw/ftw.yml"


def test_load_corpus():
    stages = ftw.load_tests([CORPUS])
    titles = {s.test for s in stages}
    assert len(titles) >= 15
    assert any(s.tx is None for s in stages)  # encoded_request is reported, not guessed
    ov = ftw.load_overrides(os.path.join(CORPUS, "ftw.yml"))
    assert "920100-4" in ov


@pytest.mark.skipif(not os.path.exists(REF_FTW), reason="reference checkout absent")
def test_reference_override_list_loads():
    ov = ftw.load_overrides(REF_FTW)
    assert len(ov) >= 50 and "911100-5" in ov


def _oracle_check(stages):
    cfg = coraza.parse_seclang(open(RULES).read())
    bad = []
    for s in stages:
        if s.tx is None:
            continue
        v = coraza.inspect(cfg, compare.oracle_request(s.tx), ())
        got = set(v.matched)
        if [x for x in s.expect_ids if x not in got] or [x for x in s.no_expect_ids if x in got]:
            bad.append((s.test, s.expect_ids, s.no_expect_ids, sorted(got)))
    return bad


def test_corpus_expectations_hold_in_the_oracle():
    ov = ftw.load_overrides(os.path.join(CORPUS, "ftw.yml"))
    stages = [s for s in ftw.load_tests([CORPUS]) if s.test not in ov]
    assert not _oracle_check(stages)


@pytest.mark.gpu
def test_gpu_ftw_replay():
    rs = gpuinspect.Ruleset(open(RULES).read())
    stages = ftw.load_tests([CORPUS])
    ov = ftw.load_overrides(os.path.join(CORPUS, "ftw.yml"))
    out = ftw.replay(rs, stages, ov)
    assert out["fail"] == 0, out["failures"]
    assert out["ignored"] == 1 and out["pass"] >= 15
    # and the verdicts are the oracle's
    run = [s for s in stages if s.tx is not None and s.test not in ov]
    batch = gpuinspect.pack([s.tx for s in run])
    res = gpuinspect.Engine(rs, matched_cap=256).inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(open(RULES).read()), batch, rs.exports)
    assert not compare.compare(res, orc)
