"""The wave-parallel body parsers of k_bparse (kernels.hip wave_parse_urlenc,
wave_parse_json) against the oracle's parse_query / json_flatten, through
rules whose exported counters see every field's key and value (counts of
non-empty / empty values, escape leftovers, exact key / value shapes, long
values).  The bodies put segment ends, '=' signs and escapes on the
boundaries the parsers cut at: 64-byte lane slices, 4 KB steps, and the
JSON parser's 4 KB LDS window and 1 KB key buffer.  A body the wave parser
does not take (k_eval parses it) gives the same verdicts, so only the
counters below tell a wrong field apart."""
import numpy as np
import pytest

import gpuinspect
from oracle import compare, coraza

RULES = """SecRuleEngine On
SecRequestBodyAccess On
SecRule REQUEST_HEADERS:Content-Type "@rx json" "id:10,phase:1,pass,nolog,ctl:requestBodyProcessor=JSON"
SecRule ARGS_POST "@rx ." "id:101,phase:2,pass,nolog,setvar:tx.nv=+1"
SecRule ARGS_POST_NAMES "@rx ." "id:102,phase:2,pass,nolog,setvar:tx.nk=+1"
SecRule ARGS_POST "@rx [ %+]" "id:103,phase:2,pass,nolog,setvar:tx.sp=+1"
SecRule ARGS_POST_NAMES "@rx [ %+=]" "id:104,phase:2,pass,nolog,setvar:tx.ks=+1"
SecRule ARGS_POST "@rx ^x{1000}" "id:105,phase:2,pass,nolog,setvar:tx.long=+1"
SecRule ARGS_POST:/^(?:json\\.)?k[0-9]+$/ "@rx ^v[0-9]+$" "id:106,phase:2,pass,nolog,setvar:tx.kv=+1"
SecRule ARGS_POST "@rx ^$" "id:107,phase:2,pass,nolog,setvar:tx.em=+1"
SecRule ARGS_POST "@rx [AB]" "id:108,phase:2,pass,nolog,setvar:tx.ab=+1"
SecRule &ARGS_POST "@gt 300" "id:109,phase:2,pass,nolog,setvar:tx.many=1"
"""
EXPORTS = ("nv", "nk", "sp", "ks", "long", "kv", "em", "ab")


def _urlenc_bodies():
    out = [b"&", b"&&a=1&&", b"=", b"a", b"a=", b"=b", b"a==b", b"%41=%42", b"a+b=c+d&%zz=%4", b"k1=v1&k2=v2&k3",
           b"x=" + b"x" * 5000, b"x" * 5000 + b"=1", b"&" * 70 + b"k7=v7"]
    for n in (63, 64, 65, 67, 68, 69, 127, 128, 4095, 4096, 4097, 4160, 8195):
        # fields whose separators fall on every offset around the lane and step cuts
        body = bytearray()
        i = 0
        while len(body) < n:
            body += b"k%d=v%d&" % (i, i)
            i += 1
        out.append(bytes(body[:n]))
    rng = np.random.Generator(np.random.PCG64(11))
    alpha = np.frombuffer(b"kv0123456789ab==&&%%++AB", dtype=np.uint8)
    for _ in range(60):
        n = int(rng.integers(1, 9000))
        out.append(alpha[rng.integers(0, len(alpha), n)].tobytes())
    for _ in range(20):  # runs of plain bytes with rare separators: segments across many lanes
        n = int(rng.integers(3000, 14000))
        b = bytearray(rng.choice(np.frombuffer(b"xxxxxxxxxxxxxxxk", dtype=np.uint8), n).tobytes())
        for p in rng.integers(0, n, 6):
            b[int(p)] = ord(rng.choice([b"&", b"=", b"%", b"+"]))
        out.append(bytes(b))
    return out


def _json_bodies():
    out = [b'{"k1": "v1", "k2": "v2", "k3": 3}',
           b'{"' + b"k" * 1100 + b'": "A"}',  # past the 1 KB key buffer
           b'{"a": {"' + b"b" * 1000 + b'": {"c": "v1"}}}']
    rng = np.random.Generator(np.random.PCG64(12))
    for _ in range(12):
        members = []
        for i in range(int(rng.integers(50, 600))):
            v = b'"v%d"' % i if i % 3 else b'"' + b"x" * int(rng.integers(0, 200)) + b'\\u0041"'
            members.append(b'"k%d": %s' % (i, v))
            if i % 17 == 0:
                members.append(b'"k%d": [1, "A+B", {"k%d": "v%d"}, []]' % (i, i, i))
        out.append(b"{" + b", ".join(members) + b"}")
    out.append(b'{"s": "' + b"x" * 9000 + b'"}')  # a string across two LDS windows
    out.append(b'{"k1": "v1", "k1": "v2", ' + b", ".join(b'"k%d": "v%d"' % (i, i) for i in range(2, 400)) +
               b', "k2": "A"}')  # repeated keys, one 400 fields apart
    return out


def _batch(bodies, ctype):
    txs = []
    for b in bodies:
        t = gpuinspect.Transaction(method=b"POST", uri=b"/submit")
        t.add_request_header("Host", "x")
        t.add_request_header("Content-Type", ctype)
        t.write_request_body(b)
        txs.append(t)
    return gpuinspect.pack(txs)


@pytest.mark.parametrize("kind", ["urlencoded", "json"])
def test_body_parser_bodies_well_formed(kind):
    """The oracle accepts every JSON body here; the urlencoded ones all
    split into fields (their counters are not all zero)."""
    if kind == "json":
        for b in _json_bodies():
            assert coraza.json_flatten(b) is not None
    else:
        assert len(_urlenc_bodies()) > 100


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["urlencoded", "json"])
def test_gpu_wave_body_parsers(kind):
    bodies = _urlenc_bodies() if kind == "urlencoded" else _json_bodies()
    ctype = "application/x-www-form-urlencoded" if kind == "urlencoded" else "application/json"
    batch = _batch(bodies, ctype)
    rs = gpuinspect.Ruleset(RULES, tx_exports=EXPORTS)
    res = gpuinspect.Engine(rs, matched_cap=128).inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(RULES), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad[:5]
    nv = sum(res.tx(i, "nv") for i in range(batch.n_req))
    assert nv > 1000
    assert sum(res.tx(i, "kv") for i in range(batch.n_req)) > 100
