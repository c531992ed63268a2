"""REQUEST_BODY links on the GPU (k_body: one wave per body, chains and
automata split over the lanes at sync points) vs the oracle's sequential
restatement.  Bodies are dense in escape sequences, entity fragments,
backslashes, whitespace runs and non-ASCII bytes so that chunk boundaries
fall next to (and inside the lookahead of) every sequence kind; the rules
cover every chunked transformation, a sequential one (t:trim), long-range
and anchored patterns, @pm / @contains / negated @rx and the @validate*
operators.  Bit-exact verdicts (matched ids, scores) are required."""
import numpy as np
import pytest

import gpuinspect
from oracle import compare, coraza

CH = "t:none,t:urlDecodeUni,t:htmlEntityDecode,t:jsDecode,t:cssDecode,t:lowercase"
RULES = """SecRuleEngine On
SecRequestBodyAccess On
SecRule REQUEST_BODY "@rx <script" "id:101,phase:2,pass,%s,setvar:tx.anomaly_score=+1"
SecRule REQUEST_BODY "@rx a[^z]{0,300}b9" "id:102,phase:2,pass,t:none,t:lowercase"
SecRule REQUEST_BODY "@rx ^zz" "id:103,phase:2,pass,t:none,t:urlDecode"
SecRule REQUEST_BODY "@rx \\bcat\\b" "id:104,phase:2,pass,t:none,t:cmdLine"
SecRule REQUEST_BODY "@rx x y;" "id:105,phase:2,pass,t:none,t:compressWhitespace"
SecRule REQUEST_BODY "@pm evil wicked" "id:106,phase:2,pass,t:none,t:urlDecodeUni,t:removeNulls"
SecRule REQUEST_BODY "@contains &amp;" "id:107,phase:2,pass,t:none"
SecRule REQUEST_BODY "!@rx q" "id:108,phase:2,pass,t:none"
SecRule REQUEST_BODY "@validateByteRange 10,32-126" "id:109,phase:2,pass,t:none"
SecRule REQUEST_BODY "@validateUrlEncoding" "id:110,phase:2,pass,t:none"
SecRule REQUEST_BODY "@validateUtf8Encoding" "id:111,phase:2,pass,t:none,t:urlDecodeUni"
SecRule REQUEST_BODY "@rx %%u00e9" "id:112,phase:2,pass,t:none,t:utf8toUnicode"
SecRule REQUEST_BODY "@rx 3c736372" "id:113,phase:2,pass,t:none,t:hexEncode"
SecRule REQUEST_BODY "@rx PHNjcmlwd" "id:114,phase:2,pass,t:none,t:base64Encode"
SecRule REQUEST_BODY "@rx \\$\\{" "id:115,phase:2,pass,t:none,t:trim,t:urlDecodeUni"
SecRule REQUEST_BODY "@rx é.{0,3}q" "id:116,phase:2,pass,t:none,t:lowercase,t:jsDecode"
SecRule REQUEST_BODY "@rx (?:a|b){3}$" "id:117,phase:2,pass,t:none,t:htmlEntityDecode"
SecRule REQUEST_BODY "@rx (?i)wicked\\+evil" "id:118,phase:2,pass,t:none,t:replaceNulls,t:compressWhitespace,t:urlEncode"
SecRule REQUEST_BODY "@rx <[a-z]" "id:119,phase:2,pass,t:none,t:cssDecode"
""" % CH

TOKENS = [b"%u0041", b"%u003c", b"%uff1c", b"%3c", b"%3C", b"%", b"%u", b"%4", b"&#x3c;", b"&#60;", b"&lt;", b"&amp;",
          b"&#x", b"&", b"&#", b"\\x3c", b"\\u003c", b"\\74", b"\\", b"\\3c ", b"\\00003c", b"<script", b"<SCRIPT",
          b"evil", b"wicked", b"wicked  \t evil", b"cat ", b" cat", b"c'a't", b"x   y;", b"x \t\n y;", b"zz", b"\nzz",
          b"a", b"b9", b"aab", b"\xc3\xa9", b"\xc3", b"\xe2\x82\xac", b"\xff", b"\x00", b"${", b" ", b"\n", b"q",
          b"PHNjcmlwd", b"+", b"=", b"&&", b";", b"\"", b"^", b",", b"(", b"/"]
FILL = np.frombuffer(b"abcdefghijklmnoprstuvwxy0123456789-_.ABCDEF", np.uint8)


def bodies(n, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        target = int(rng.integers(60, 9000)) if i % 4 else int(rng.integers(1, 300))
        parts = []
        size = 0
        while size < target:
            if rng.random() < 0.35:
                t = TOKENS[int(rng.integers(0, len(TOKENS)))]
            else:
                t = FILL[rng.integers(0, len(FILL), int(rng.integers(1, 40)))].tobytes()
            parts.append(t)
            size += len(t)
        out.append(b"".join(parts))
    # escape sequences straddling every lane boundary of a 64-lane split
    for L in (64, 128, 640, 6400):
        for tok in (b"%u003c", b"&#x3c;", b"\\u003c", b"\\00003c ", b"<script", b"wicked \t evil", b"\xe2\x82\xac"):
            for d in range(len(tok) + 1):
                b = bytearray(b"k" * L)
                for j in range(1, 64):
                    p = L * j // 64 - d
                    if 0 <= p and p + len(tok) <= L:
                        b[p:p + len(tok)] = tok
                out.append(bytes(b))
    return out


def tile_edge_bodies():
    """Stretches longer than k_body's 3 KB LDS tile without a sync point of
    some transformation (lane 0 then runs to the next one), and sequences
    straddling the tile boundaries."""
    return [b"k" * 7000 + b"&lt;script", b"%" * 7000 + b"3cscript", b"\\" * 5001 + b"u003cscript",
            b"ab%u003c" * 1500, b"&#x3c;script " * 900, (b"%u003c" + b"k" * 3066) * 3 + b"script"]


def batch_of(bs):
    txs = []
    for b in bs:
        t = gpuinspect.Transaction(method=b"POST", uri=b"/form")
        t.add_request_header("Host", "x")
        t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
        t.write_request_body(b)
        txs.append(t)
    return gpuinspect.pack(txs)


def test_oracle_rules_parse():
    coraza.parse_seclang(RULES)
    gpuinspect.Ruleset(RULES)


def _parity(bs):
    batch = batch_of(bs)
    rs = gpuinspect.Ruleset(RULES)
    res = gpuinspect.Engine(rs).inspect(batch)
    cfg = coraza.parse_seclang(RULES)
    verdicts = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:5]
    return verdicts


@pytest.mark.gpu
def test_gpu_body_chunks_tile_edges():
    _parity(tile_edge_bodies() + bodies(8, seed=3))


@pytest.mark.gpu
def test_gpu_body_chunks_parity():
    verdicts = _parity(bodies(500))
    # the rules do fire (the test is not vacuous)
    fired = {}
    for v in verdicts.values():
        for m in v.matched:
            fired[m] = fired.get(m, 0) + 1
    for rid in range(101, 120):
        assert fired.get(rid, 0) > 0, (rid, fired)
