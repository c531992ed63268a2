"""JSON request bodies (ctl:requestBodyProcessor=JSON -> ARGS_POST).

CPU: the oracle's restatement of coraza internal/bodyprocessors/json.go
(readItems over tidwall/gjson v1.18.0) on hand-checked vectors.  coraza is
not vendored under /root/reference and no Go toolchain is here, so these
vectors restate the upstream behaviour documented in json.go's own comment
("json.data.name", "json.items.0", and "json.items" = the element count);
they are parity-unpinned beyond that (Oracle).

GPU: the HIP body processor vs the oracle, bit-exact verdicts, on edge-case
bodies and on the C3 traffic mix.
"""
import os

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRS = os.path.join(ROOT, "rulesets", "crs_pl1.conf")

VECTORS = [
    # json.go readItems comment examples
    (b'{"data": {"name": "John", "age": 30}, "items": [1,2,3]}',
     [(b"json.data.name", b"John"), (b"json.data.age", b"30"), (b"json.items.0", b"1"),
      (b"json.items.1", b"2"), (b"json.items.2", b"3"), (b"json.items", b"3")]),
    (b'[{"data": {"name": "John", "age": 30}, "items": [1,2,3]}]',
     [(b"json.0.data.name", b"John"), (b"json.0.data.age", b"30"), (b"json.0.items.0", b"1"),
      (b"json.0.items.1", b"2"), (b"json.0.items.2", b"3"), (b"json.0.items", b"3"), (b"json", b"1")]),
    # scalars: raw numbers / booleans, null -> ""
    (b'{"a": -1.50e+3, "b": true, "c": false, "d": null, "e": 0}',
     [(b"json.a", b"-1.50e+3"), (b"json.b", b"true"), (b"json.c", b"false"), (b"json.d", b""), (b"json.e", b"0")]),
    # empty containers write nothing
    (b'{"a": {}, "b": [], "c": [[]]}', [(b"json.c", b"1")]),
    (b"{}", []),
    (b" [ ] ", []),
    # escapes in values and keys; surrogate pairs; lone surrogates -> U+FFFD
    (b'{"k\\"ey": "a\\n\\t\\/\\\\b", "u": "\\u00e9\\u20ac", "p": "\\ud83d\\ude00", "l": "\\ud800x", "m": "\\ud800\\u0041"}',
     [(b'json.k"ey', b"a\n\t/\\b"), (b"json.u", "é€".encode()), (b"json.p", "\U0001F600".encode()),
      (b"json.l", b"\xef\xbf\xbdx"), (b"json.m", b"\xef\xbf\xbd")]),
    # a repeated key: first position, last value
    (b'{"a": 1, "b": 2, "a": 3}', [(b"json.a", b"3"), (b"json.b", b"2")]),
    (b'{"a": [5, 6], "a.0": 7}', [(b"json.a.0", b"7"), (b"json.a.1", b"6"), (b"json.a", b"2")]),
    # keys are case-sensitive
    (b'{"A": 1, "a": 2}', [(b"json.A", b"1"), (b"json.a", b"2")]),
    # raw UTF-8 passes through
    ('{"café": "ü"}'.encode(), [("json.café".encode(), "ü".encode())]),
]

SCALAR_ROOTS = [b"1", b'"s"', b"null", b" -2 "]  # engine limit: flagged unsupported
INVALID = [b"", b"  ", b"x", b"{", b'{"a":1,}', b"[1,]", b"[01]", b"[1.]", b"[.5]", b"[-]",
           b"[1e]", b'{"a" 1}', b"{a:1}", b"[tru]", b"[nul]", b'["\\x"]', b'["\\u12"]', b'["a\nb"]',
           b"[1] x", b"[1][2]", b"{'a':1}", b"[1 2]", b'{"a":1 "b":2}']


@pytest.mark.parametrize("body,want", VECTORS, ids=[str(i) for i in range(len(VECTORS))])
def test_oracle_json_flatten(body, want):
    assert coraza.json_flatten(body) == want


@pytest.mark.parametrize("body", INVALID, ids=[str(i) for i in range(len(INVALID))])
def test_oracle_json_invalid(body):
    """Not JSON: readJSON's error -> REQBODY_ERROR (not an engine limit)."""
    with pytest.raises(coraza.JsonBodyError):
        coraza.json_flatten(body)


@pytest.mark.parametrize("body", SCALAR_ROOTS, ids=[str(i) for i in range(len(SCALAR_ROOTS))])
def test_oracle_json_scalar_root(body):
    assert coraza.json_flatten(body) is None


def test_oracle_json_first_event_decides():
    """Left to right, the first of {syntax error, engine limit} decides."""
    deep_then_bad = b"[" * (coraza.JSON_MAX_DEPTH + 1) + b"x"
    assert coraza.json_flatten(deep_then_bad) is None
    bad_then_deep = b"[x" + b"[" * (coraza.JSON_MAX_DEPTH + 1)
    with pytest.raises(coraza.JsonBodyError):
        coraza.json_flatten(bad_then_deep)


def test_oracle_json_body_error_verdict():
    """CRS base rule 200002 (REQBODY_ERROR !@eq 0 -> deny 400,
    generate_coreruleset_configmaps.py:73-81) fires on a body that is not JSON."""
    cfg = coraza.parse_seclang(open(CRS).read())
    req = coraza.Request(b"POST", b"/api", b"HTTP/1.1", [(b"Host", b"x"), (b"Content-Type", b"application/json")],
                         b'{"a": 1,}')
    v = coraza.inspect(cfg, req)
    assert not v.unsupported and (v.rule_id, v.status, v.phase) == (200002, 400, 2)
    ok = coraza.Request(b"POST", b"/api", b"HTTP/1.1", [(b"Host", b"x"), (b"Content-Type", b"application/json")],
                        b'{"a": 1}')
    assert coraza.inspect(cfg, ok).status == 0


def test_oracle_json_depth_limit():
    ok = b"[" * coraza.JSON_MAX_DEPTH + b"]" * coraza.JSON_MAX_DEPTH + b" " * 1000  # room for the keys
    deep = b"[" * (coraza.JSON_MAX_DEPTH + 1) + b"]" * (coraza.JSON_MAX_DEPTH + 1)
    got = coraza.json_flatten(ok)  # every array but the innermost holds one element
    assert len(got) == coraza.JSON_MAX_DEPTH - 1 and all(v == b"1" for _, v in got)
    assert coraza.json_flatten(deep) is None
    one = b"[" * coraza.JSON_MAX_DEPTH + b"1" + b"]" * coraza.JSON_MAX_DEPTH
    assert coraza.json_flatten(one) is None  # 4480 flattened key bytes > 4 x 129 + 1024
    got = coraza.json_flatten(one + b" " * 1000)
    assert got[0] == (b"json" + b".0" * coraza.JSON_MAX_DEPTH, b"1") and len(got) == coraza.JSON_MAX_DEPTH + 1


def test_generator_json_bodies_valid():
    g = traffic.TrafficGen(traffic.SEED + 7)
    for k in range(20):
        b = g._json_body(k % 3 == 0)
        assert 4096 <= len(b) <= 65536 + 400
        assert coraza.json_flatten(b), b[:80]


def _json_tx(body, ctype=b"application/json", uri=b"/api/v1/users"):
    t = gpuinspect.Transaction(method=b"POST", uri=uri)
    t.add_request_header("Host", "api.example.com")
    t.add_request_header("Content-Type", ctype)
    t.write_request_body(body)
    return t


def _parity(text, batch):
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    return res, orc


@pytest.mark.gpu
def test_gpu_json_edge_bodies():
    text = open(CRS).read()
    bodies = [b for b, _ in VECTORS] + INVALID + SCALAR_ROOTS
    deep = b"[" * 64 + b'"<script>alert(1)</script>"' + b"]" * 64
    bodies += [deep, deep + b" " * 1100, b"[" * 65 + b"]" * 65,
               b'{"q": "1 UNION SELECT username, password FROM users"}',
               b'{"a": {"b": ["<script>alert(1)</script>", {"c": "../../../../etc/passwd"}]}}',
               b'{"x\\u003cscript\\u003e": "evilmonkey", "cmd": ";cat /etc/passwd"}',
               b'{"s": "\\u003cimg src=x onerror=alert(1)\\u003e"}',
               b'{"a": "' + b"A" * 5000 + b'", "b": [' + b",".join(b"%d" % i for i in range(2000)) + b"]}",
               b'[' + b",".join(b'{"k":"v%d","k":"w%d"}' % (i, i) for i in range(300)) + b"]",
               b"\n\t {\"ws\" : [ 1 , 2 ] } \r\n",
               # wave_parse_json: a key past its 1 KB path buffer (k_eval parses the body), keys and
               # escaped strings across its 4 KB LDS windows, a repeated key 200 fields apart
               b'{"' + b"k" * 1500 + b'": 1, "x": "<script>alert(1)</script>"}',
               b'{' + b",".join(b'"f\\u00e9%d": "v\\n%s"' % (i, b"x" * (i % 97)) for i in range(400)) + b'}',
               b'{"d": 1, ' + b",".join(b'"e%d": [%d, "s"]' % (i, i) for i in range(200)) + b', "d": "<script>"}']
    txs = [_json_tx(b) for b in bodies]
    txs += [_json_tx(b, ctype=b"application/vnd.api+json") for b in bodies[:4]]
    res, orc = _parity(text, gpuinspect.pack(txs))
    # bodies that are not JSON get Coraza's verdict: REQBODY_ERROR -> rule 200002 -> 400
    nv = len(VECTORS)
    # (an empty body is never processed: ProcessRequestBody skips empty bodies)
    for k in range(nv, nv + len(INVALID)):
        want = (200002, 400) if bodies[k] else (0, 0)
        assert (int(res.verdicts[k]["rule_id"]), int(res.verdicts[k]["status"])) == want, bodies[k]
        assert bool(int(res.verdicts[k]["flags"]) & gpuinspect.GI_REQ_BODY_ERROR) == bool(bodies[k])
    # engine limits (scalar roots, nesting deeper than 64) stay flagged
    assert all(int(res.verdicts[k]["flags"]) & gpuinspect.GI_REQ_UNSUPPORTED_BODY
               for k in range(nv + len(INVALID), nv + len(INVALID) + len(SCALAR_ROOTS)))
    assert sum(1 for o in orc.values() if o.unsupported) == len(SCALAR_ROOTS) + 2  # + 65 deep, + 64 deep w/o room
    assert int((res.verdicts["action"] != 0).sum()) >= 5 + len(INVALID) - 1


@pytest.mark.gpu
def test_gpu_parity_c3_json_mix():
    text = open(CRS).read()
    batch = traffic.TrafficGen(traffic.SEED + 3).batch(48, post_frac=0.8, attack_rate=0.3, json_frac=0.6)
    res, orc = _parity(text, batch)
    assert not any(o.unsupported for o in orc.values())
    assert int((res.verdicts["action"] != 0).sum()) > 5
