"""MATCHED_VARS over long capture groups and expanded values (ADVICE r04,
low): TX.0 / TX.1 hold captures of multi-KB values, one of them hex-encoded
(2x the value), and a later rule's MATCHED_VARS / MATCHED_VAR copy them.  The
matched-variable arena is sized for the capture groups (runtime.cpp
request_layout: cap_groups x cap_t), so the GPU must neither overflow nor
differ from the oracle, which has no such limit.  (A setvar that copies
such a value into a TX string is bounded by the TX string arena instead:
past it the request is flagged unsupported, never answered wrongly --
DESIGN.md section 9.)"""
import pytest

import gpuinspect
from oracle import compare, coraza

RULES = r"""SecRuleEngine On
SecRequestBodyAccess On
SecRule ARGS:a "@rx ^(x+)(y*)$" "id:10,phase:2,pass,capture,t:none,setvar:tx.c=1"
SecRule ARGS:b "@rx ^(.+)$" "id:11,phase:2,pass,capture,t:none,t:hexEncode,setvar:tx.d=1"
SecRule TX:0|TX:1|TX:2 "@rx ^(?:x{64}|(?:3[0-9]){64})" "id:20,phase:2,pass,chain,setvar:tx.score=+1"
    SecRule MATCHED_VARS "@rx (?:xxxx|3[0-9]3[0-9])$" "setvar:tx.score=+10"
SecRule MATCHED_VAR "@rx ^(?:x|3)" "id:21,phase:2,pass,setvar:tx.score=+100"
SecRule MATCHED_VARS_NAMES "@rx ^TX:" "id:22,phase:2,pass,setvar:tx.score=+1000"
SecRule TX:SCORE "@ge 1000000" "id:949,phase:2,deny,status:403"
"""


def batch():
    txs = []
    for n in (10, 600, 3000, 9000):  # (operators stay small automata: the copies are what is long)
        for body in (b"a=" + b"x" * n + b"y" * (n // 3), b"b=" + b"0123456789" * (n // 10 + 1),
                     b"a=" + b"x" * n + b"&b=" + b"9" * n):
            t = gpuinspect.Transaction(method=b"POST", uri=b"/p")
            t.add_request_header("Host", "x")
            t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
            t.write_request_body(body)
            txs.append(t)
    return gpuinspect.pack(txs)


def test_oracle_long_matched_vars():
    cfg = coraza.parse_seclang(RULES)
    b = batch()
    rs = gpuinspect.Ruleset(RULES)
    v = compare.oracle_verdicts(cfg, b, rs.exports)
    assert any(20 in x.matched and 21 in x.matched for x in v.values())  # long copies do happen


@pytest.mark.gpu
def test_gpu_long_matched_vars():
    b = batch()
    rs = gpuinspect.Ruleset(RULES)
    res = gpuinspect.Engine(rs).inspect(b)
    bad = compare.compare(res, compare.oracle_verdicts(coraza.parse_seclang(RULES), b, rs.exports))
    assert not bad, bad[:4]
    assert not (res.verdicts["flags"] & 0x0F).any(), [int(f) for f in res.verdicts["flags"]]  # no overflow
