"""ctl:ruleRemoveTargetById [upstream coraza internal/actions/ctl.go,
rule.go doEvaluate: the removed (variable, key) pairs become exceptions of
the rule's variables for the rest of the transaction; a single's key is ""].
CPU: the oracle on hand-checked cases; GPU: kernels.hip target_removed vs the
oracle, bit-exact."""
import pytest

import gpuinspect
from oracle import compare, coraza

RULES = """SecRuleEngine On
SecRule ARGS:skip "@streq 1" "id:10,phase:1,pass,nolog,ctl:ruleRemoveTargetById=100;ARGS:pw,ctl:ruleRemoveTargetById=101-102;REQUEST_HEADERS:x-a,ctl:ruleRemoveTargetById=103;REQUEST_URI"
SecRule ARGS "@rx evil" "id:100,phase:2,pass,setvar:tx.anomaly_score=+1"
SecRule REQUEST_HEADERS "@rx evil" "id:101,phase:2,pass,setvar:tx.anomaly_score=+10"
SecRule &REQUEST_HEADERS:x-a "@eq 1" "id:102,phase:2,pass,setvar:tx.anomaly_score=+100"
SecRule REQUEST_URI "@rx evil" "id:103,phase:2,pass,setvar:tx.anomaly_score=+1000"
SecRule ARGS_NAMES "@rx ^pw$" "id:104,phase:2,pass,setvar:tx.anomaly_score=+10000"
SecRule ARGS:pw "@rx evil" "id:105,phase:2,pass,setvar:tx.anomaly_score=+100000"
"""

CASES = [  # (uri, headers, expected matched ids)
    (b"/?pw=evil", [(b"X-A", b"evil")], [100, 101, 102, 103, 104, 105]),
    (b"/?skip=1&pw=evil", [(b"X-A", b"evil")], [104, 105]),
    (b"/?skip=1&pw=evil&q=evil", [(b"X-A", b"evil"), (b"X-B", b"evil")], [100, 101, 104, 105]),
    (b"/evil?skip=1", [], []),
    (b"/evil?skip=0", [], [103]),
    (b"/?skip=1&PW=evil", [(b"x-a", b"ok")], []),  # the removal compares lowercased keys: "PW" is removed too
]


def _batch(cases):
    txs = []
    for uri, hdrs, _ in cases:
        t = gpuinspect.Transaction(method=b"GET", uri=uri)
        t.add_request_header("Host", "x")
        for k, v in hdrs:
            t.add_request_header(k, v)
        txs.append(t)
    return gpuinspect.pack(txs)


def test_compile_ctl_targets():
    gpuinspect.Ruleset(RULES)


@pytest.mark.parametrize("k", range(len(CASES)))
def test_oracle_ctl_targets(k):
    cfg = coraza.parse_seclang(RULES)
    b = _batch([CASES[k]])
    v = compare.oracle_verdicts(cfg, b, gpuinspect.DEFAULT_EXPORTS)[0]
    assert [m for m in v.matched if m != 10] == CASES[k][2]


@pytest.mark.gpu
def test_gpu_ctl_targets_parity():
    b = _batch(CASES * 50)
    rs = gpuinspect.Ruleset(RULES)
    res = gpuinspect.Engine(rs).inspect(b)
    cfg = coraza.parse_seclang(RULES)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, b, rs.exports))
    assert not bad, bad[:5]
