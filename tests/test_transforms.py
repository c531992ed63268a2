"""Transformations beyond the round-1 set: base64Decode(Ext), base64Encode,
hexDecode, hexEncode, sha1, md5, urlEncode, cssDecode, escapeSeqDecode,
removeCommentsChar ([upstream coraza internal/transformations/*.go, ported
from ModSecurity]; coraza is not vendored here: the decoders' edge cases are
parity unpinned, the digests and encoders are pinned by their RFC vectors).

CPU: the oracle on known-answer vectors.  GPU: for every (transformation,
value) pair a rule `@streq <hex of the oracle's output>` over
`t:<name>,t:hexEncode` must match on the device exactly when it does in the
oracle (the matched-rule lists are compared), plus a few chains.
"""
import pytest

import gpuinspect
from oracle import compare, coraza

KAT = [
    ("sha1", b"", bytes.fromhex("da39a3ee5e6b4b0d3255bfef95601890afd80709")),
    ("sha1", b"abc", bytes.fromhex("a9993e364706816aba3e25717850c26c9cd0d89d")),
    ("md5", b"", bytes.fromhex("d41d8cd98f00b204e9800998ecf8427e")),
    ("md5", b"abc", bytes.fromhex("900150983cd24fb0d6963f7d28e17f72")),
    ("hexencode", b"Hi\x00\xff", b"486900ff"),
    ("hexdecode", b"486900ff", b"Hi\x00\xff"),
    ("hexdecode", b"48690", b"48690"),          # odd length: error, value kept
    ("hexdecode", b"zz", b"zz"),                # non-hex: error, value kept
    ("base64encode", b"Hello", b"SGVsbG8="),
    ("base64decode", b"SGVsbG8gd29ybGQ=", b"Hello world"),
    ("base64decode", b"SGVs\r\nbG8", b"Hello"),    # CR/LF skipped
    ("base64decode", b"SGVs bG8", b"Hel"),          # stops at ' '
    ("base64decode", b"SGVsbA", b"Hell"),           # unpadded tail
    ("base64decodeext", b"SG Vs*bG8=", b"Hello"),   # invalid bytes skipped
    ("urlencode", b"a b*<~", b"a+b*%3c%7e"),
    ("cssdecode", b"\\3c script\\3E", b"<script>"),
    ("cssdecode", b"a\\\nb\\", b"ab"),
    ("cssdecode", b"\\ff1c", b"\x3c"),              # 4 digits: full-width ff1c -> '<'
    ("escapeseqdecode", b"\\x41\\101\\n\\q", b"AA\nq"),
    ("removecommentschar", b"a/*b*/c--d#e<!--f-->", b"abcdef"),
]


@pytest.mark.parametrize("name,inp,want", KAT, ids=["%s-%d" % (k[0], i) for i, k in enumerate(KAT)])
def test_oracle_transform_kat(name, inp, want):
    assert coraza.TRANSFORM_FNS[name](inp) == want


NEW = ["base64decode", "base64decodeext", "base64encode", "hexdecode", "hexencode", "sha1", "md5", "urlencode",
       "cssdecode", "escapeseqdecode", "removecommentschar"]
VALUES = [b"", b"abc", b"SGVsbG8gd29ybGQ=", b"PHNjcmlwdD5hbGVydCgxKTwvc2NyaXB0Pg", b"3c7363726970743e",
          b"\\3c script\\3e alert(1)", b"\\x3c\\163cript\\x3e", b"1/**/union/**/select--x#y",
          b"a b+c%41<>\"'", b"\\0000ff1c\\00ff1c\\ff1cz", b"A" * 200, b"ab\\", b"\\", b"x\\x4", b"SGV*sb G8="]


def _uri_escape(v: bytes) -> bytes:
    return b"".join(b"%%%02X" % c for c in v)


def _rules():
    lines = ["SecRuleEngine On", "SecRequestBodyAccess On"]
    rid = 1000
    expect = {}
    for t in NEW:
        for k, v in enumerate(VALUES):
            want = coraza.TRANSFORM_FNS[t](v).hex()
            if not want:
                continue  # @streq "" is not expressible; covered by the non-empty cases
            lines.append('SecRule ARGS_GET:v%d "@streq %s" "id:%d,phase:1,pass,nolog,t:none,t:%s,t:hexEncode"'
                         % (k, want, rid, t))
            expect[rid] = (t, v)
            rid += 1
    # chains mixing old and new transformations, and a digest feeding @rx
    lines.append('SecRule ARGS_GET "@rx (?i)<script" "id:900,phase:1,pass,t:none,t:base64Decode,t:lowercase"')
    lines.append('SecRule ARGS_GET "@rx ^[0-9a-f]{40}$" "id:901,phase:1,pass,t:none,t:sha1,t:hexEncode"')
    lines.append('SecRule ARGS_GET "@contains <script>" "id:902,phase:1,pass,t:none,t:hexDecode,t:cssDecode"')
    lines.append('SecRule ARGS_GET "@rx union\\s*select" "id:903,phase:1,pass,t:none,t:removeCommentsChar,t:urlDecodeUni"')
    return "\n".join(lines) + "\n", expect


def test_compile_new_transforms():
    text, expect = _rules()
    assert len(expect) > 100
    gpuinspect.Ruleset(text)  # every name compiles
    coraza.parse_seclang(text)  # and the oracle accepts them


@pytest.mark.gpu
def test_gpu_new_transforms():
    text, expect = _rules()
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=512)
    q = b"&".join(b"v%d=%s" % (k, _uri_escape(v)) for k, v in enumerate(VALUES))
    txs = [gpuinspect.Transaction(method=b"GET", uri=b"/?" + q)]
    for k, v in enumerate(VALUES):  # one value per request as well (every rule's own request)
        txs.append(gpuinspect.Transaction(method=b"GET", uri=b"/?v%d=%s" % (k, _uri_escape(v))))
    batch = gpuinspect.pack(txs)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    # the oracle matched every @streq rule on request 0: so did the device
    got = set(res.matched_rules(0))
    assert set(expect) <= got, sorted(set(expect) - got)[:10]
    assert {901} <= got
