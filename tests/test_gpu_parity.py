"""GPU parity: the HIP engine vs the CPU oracle (bit-exact verdicts).

* the reference's own KATs (tests/golden/kats.json);
* config 1 (config/samples RuleSet) over seeded synthetic traffic;
* the CRS-shaped PL1 ruleset over seeded synthetic traffic.
"""
import json
import os

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
KATS = json.load(open(os.path.join(GOLDEN, "kats.json")))

pytestmark = pytest.mark.gpu


def _tx(r):
    t = gpuinspect.Transaction()
    t.process_uri(r["uri"], r["method"], r["proto"])
    for k, v in r["headers"]:
        t.add_request_header(k, v)
    t.write_request_body(r["body"])
    return t


@pytest.mark.parametrize("sc", KATS["scenarios"], ids=[s["name"] for s in KATS["scenarios"]])
def test_gpu_kats(sc):
    rs = gpuinspect.Ruleset(gpuinspect.aggregate_configmaps(sc["configmaps"]))
    eng = gpuinspect.Engine(rs)
    res = eng.inspect([_tx(r) for r in sc["requests"]])
    for i, r in enumerate(sc["requests"]):
        it = res.interruption(i)
        status = it["status"] if it else 200
        assert status == r["expect_status"], (r["source"], r["uri"], it)
        m = res.matched_rules(i)
        for x in r["expect_matched"]:
            assert x in m, (r["source"], m)
        for x in r["expect_not_matched"]:
            assert x not in m, (r["source"], m)


def _parity(text, batch, n_check=None):
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    res = eng.inspect(batch)
    cfg = coraza.parse_seclang(text)
    idx = range(batch.n_req) if n_check is None else range(min(n_check, batch.n_req))
    orc = compare.oracle_verdicts(cfg, batch, rs.exports, idx)
    bad = compare.compare(res, orc)
    assert not bad, bad
    return res


def test_gpu_parity_samples_c1():
    text = open(os.path.join(GOLDEN, "samples_ruleset.conf")).read()
    batch = traffic.TrafficGen(traffic.SEED).batch(3000, attack_rate=0.3)
    res = _parity(text, batch)
    assert int(res.verdicts["match_cnt"].astype(bool).sum()) > 50  # attacks were seen


def test_gpu_parity_edge_uris():
    text = open(os.path.join(GOLDEN, "samples_ruleset.conf")).read()
    uris = [b"/", b"*", b"/a b?x=1", b"/%zz?q=evilmonkey", b"/p%41th?a=%u0041&b=%uFF1Cscript%uFF1E",
            b"/x?", b"/x??a=1", b"/x#frag?q=evilmonkey", b"//double?q=1", b"http://h/x",
            b"/\x01ctl?q=evilmonkey", b"/caf\xc3\xa9?q=<script>alert(1)</script>",
            b"/?q=select+*+from+users", b"/?=evilmonkey&&&a", b"/?q=%3Cscript%3E", b"/\xff\xfe?x=1"]
    txs = []
    for u in uris:
        t = gpuinspect.Transaction(method=b"GET", uri=u)
        t.add_request_header("Host", "x")
        t.add_request_header("Cookie", " a=1; b ; =c;d=evilmonkey ")
        txs.append(t)
    res = _parity(text, gpuinspect.pack(txs))
    # every request-target form (absolute, scheme-relative, "*", control bytes)
    # is evaluated: none is flagged unsupported on either side
    assert not (res.verdicts["flags"] & 0x0F).any(), [int(f) for f in res.verdicts["flags"]]


CRS = os.path.join(ROOT, "rulesets", "crs_pl1.conf")


def test_gpu_parity_crs_pl1_get():
    text = open(CRS).read()
    batch = traffic.TrafficGen(traffic.SEED + 1).batch(1500, attack_rate=0.3)
    res = _parity(text, batch)
    assert int((res.verdicts["action"] != 0).sum()) > 50


def test_gpu_parity_crs_pl1_mixed_post():
    text = open(CRS).read()
    batch = traffic.TrafficGen(traffic.SEED + 2).batch(200, post_frac=0.5, attack_rate=0.3)
    _parity(text, batch)


def test_gpu_parity_crs_pl4_c3_mix():
    """C4's ruleset (blocking paranoia level 4, the PL2-4 rules and
    libinjection at PL1) over the C3 request mix."""
    text = open(os.path.join(ROOT, "rulesets", "crs_pl4.conf")).read()
    batch = traffic.TrafficGen(traffic.SEED + 4).batch(300, post_frac=0.5, attack_rate=0.3)
    res = _parity(text, batch)
    assert int((res.verdicts["action"] != 0).sum()) > 30


def test_gpu_parity_crs_ftw_detection_only():
    """The go-ftw configuration (X-CRS-Test rule block, generate_coreruleset_configmaps.py:113-141):
    DetectionOnly, so nothing is interrupted, but the matched ids are compared."""
    text = open(os.path.join(ROOT, "rulesets", "crs_ftw.conf")).read()
    batch = traffic.TrafficGen(traffic.SEED + 5).batch(300, attack_rate=0.5)
    res = _parity(text, batch)
    assert int((res.verdicts["action"] != 0).sum()) == 0


def test_gpu_parity_crs_pl1_kat_payloads():
    """Every attack payload of the generator, raw and encoded, in every
    position the CRS-shaped rules look at."""
    text = open(CRS).read()
    txs = []
    for p in traffic.ATTACKS + [b"<script>alert(1)</script>", b"1 UNION SELECT username FROM users"]:
        for enc in (False, True):
            q = traffic._quote(p, enc)
            t = gpuinspect.Transaction(method=b"GET", uri=b"/search?q=" + q)
            t.add_request_header("Host", "www.example.com")
            t.add_request_header("User-Agent", p)
            t.add_request_header("Cookie", b"sid=" + q)
            txs.append(t)
            t2 = gpuinspect.Transaction(method=b"POST", uri=b"/form")
            t2.add_request_header("Host", "www.example.com")
            t2.add_request_header("Content-Type", "application/x-www-form-urlencoded")
            t2.write_request_body(b"a=1&" + q + b"=x&b=" + q)
            txs.append(t2)
    _parity(text, gpuinspect.pack(txs))


GATED = """SecRuleEngine On
SecAction "id:1,phase:1,pass,nolog,setvar:tx.pl=1"
SecRule REQUEST_HEADERS:X-Open "@streq yes" "id:2,phase:1,pass,nolog,ctl:ruleRemoveById=10"
SecRule TX:PL "@lt 2" "id:10,phase:1,pass,nolog,skipAfter:END-PL2"
SecRule ARGS "@rx evil" "id:11,phase:1,deny,status:403"
SecMarker END-PL2
SecRule ARGS "@rx monkey" "id:12,phase:1,deny,status:403"
"""


def test_gpu_parity_gated_region_reached():
    """Rule 11 sits behind a paranoia-style gate the compiler keeps out of
    phase A; a request that removes the gate (ctl:ruleRemoveById) reaches it
    and must still be evaluated exactly."""
    assert gpuinspect.Ruleset(GATED).info["n_hit_slots"] == 1  # only rule 12 is scanned
    txs = []
    for uri in (b"/?a=evil", b"/?a=monkey", b"/?a=safe"):
        for open_ in (False, True):
            t = gpuinspect.Transaction(method=b"GET", uri=uri)
            t.add_request_header("Host", "x")
            if open_:
                t.add_request_header("X-Open", "yes")
            txs.append(t)
    res = _parity(GATED, gpuinspect.pack(txs))
    assert [int(v["status"]) for v in res.verdicts] == [0, 403, 403, 403, 0, 0]


CAPTURE = """SecRuleEngine On
SecRule ARGS|REQUEST_HEADERS:User-Agent "@rx (?i)(union)\\s+(select)" "id:1,phase:2,pass,capture,t:none,t:urlDecodeUni,\\
    logdata:'Matched Data: %{TX.0} found within %{MATCHED_VAR_NAME}',setvar:'tx.anomaly_score=+5'"
SecRule ARGS "@pm evilmonkey sinister" "id:2,phase:2,pass,capture,t:lowercase,setvar:'tx.anomaly_score=+3'"
SecRule TX:ANOMALY_SCORE "@ge 5" "id:3,phase:2,deny,status:403"
"""


def test_gpu_parity_capture_logdata_only():
    """capture feeding only logdata (the CRS pattern) is dropped by the compiler;
    verdicts, matched ids and scores stay identical to the oracle, which runs
    the capture (FindStringSubmatch / phrase captures into TX.0-TX.9)."""
    txs = []
    for q in (b"1+UNION+SELECT+x", b"a%20union%20%20select", b"EvilMonkey", b"safe", b"sinister+union+select"):
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?q=" + q)
        t.add_request_header("Host", "x")
        t.add_request_header("User-Agent", "Mozilla/5.0")
        txs.append(t)
    res = _parity(CAPTURE, gpuinspect.pack(txs))
    assert [int(v["status"]) for v in res.verdicts] == [403, 403, 0, 0, 403]


PMF_RULES = """SecRuleEngine On
SecRule ARGS|REQUEST_HEADERS:User-Agent "@pmFromFile scanners.data" "id:10,phase:2,deny,status:403,t:none,t:lowercase"
SecRule ARGS_NAMES "!@pmFromFile allow.data" "id:11,phase:2,pass"
SecRule ARGS "@pmFromFile empty.data" "id:12,phase:2,deny,status:403"
"""
PMF_FILES = {
    "scanners.data": b"# scanner user agents\r\nNikto\r\n  sqlmap  \n\n#comment\nunion select\nEvil Monkey",
    "allow.data": b"q\nid\n",
    "empty.data": b"# nothing\n\n",
}


def test_gpu_parity_pmfromfile():
    """@pmFromFile (coraza pm_from_file.go): phrases from a caller-supplied
    data file, the same ASCII case-insensitive matcher as @pm, phase-A
    scanned; GPU vs oracle over seeded traffic plus targeted values."""
    rs = gpuinspect.Ruleset(PMF_RULES, data_files=PMF_FILES)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    txs = []
    for q in (b"q=NIKTO", b"id=1+UNION+SELECT+2", b"q=evil%20monkey", b"q=safe", b"x=1", b"q=sqlmap&id=2", b"q="):
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?" + q)
        t.add_request_header("Host", "x")
        t.add_request_header("User-Agent", "Mozilla/5.0")
        txs.append(t)
    t = gpuinspect.Transaction(method=b"GET", uri=b"/")
    t.add_request_header("User-Agent", "sqlmap/1.7")
    txs.append(t)
    batch = gpuinspect.pack(txs)
    res = eng.inspect(batch)
    cfg = coraza.parse_seclang(PMF_RULES, PMF_FILES)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, batch, rs.exports, range(batch.n_req)))
    assert not bad, bad
    assert [int(v["status"]) for v in res.verdicts] == [403, 403, 403, 0, 0, 403, 0, 403]
    big = traffic.TrafficGen(traffic.SEED + 7).batch(1000, attack_rate=0.3)
    res = eng.inspect(big)
    bad = compare.compare(res, compare.oracle_verdicts(cfg, big, rs.exports, range(big.n_req)))
    assert not bad, bad


MULTI = """SecRuleEngine On
SecRule ARGS "@rx ^abc$" "id:1,phase:2,pass,multiMatch,t:lowercase,setvar:'tx.anomaly_score=+1'"
SecRule ARGS "@contains %3c" "id:2,phase:2,pass,multiMatch,t:none,t:urlDecodeUni,t:lowercase,setvar:'tx.anomaly_score=+10'"
SecRule ARGS|REQUEST_HEADERS:User-Agent "@rx <script" "id:3,phase:2,pass,multiMatch,t:urlDecodeUni,t:htmlEntityDecode,setvar:'tx.anomaly_score=+100'"
SecRule ARGS "@rx ^abc$" "id:4,phase:2,pass,t:lowercase,setvar:'tx.anomaly_score=+1000'"
SecRule TX:ANOMALY_SCORE "@ge 1002" "id:9,phase:2,deny,status:403"
"""


def test_gpu_parity_multimatch():
    """multiMatch (rule.go executeTransformationsMultimatch): the operator runs
    on the raw value and after every transformation that changed the value,
    each match counting (and running setvar) once; interpreter-only links.
    The exported anomaly_score pins the match counts: a=ABC matches rule 1
    once (after t:lowercase), a=abc once (raw; lowercase is a no-op and adds
    no candidate), so neither reaches 1002; GPU vs oracle."""
    txs = []
    for q in (b"a=ABC", b"a=abc", b"a=%253c", b"a=%253C", b"a=%253Cscript", b"a=%26lt;script", b"a=safe", b"a=abc&b=ABC"):
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?" + q)
        t.add_request_header("Host", "x")
        t.add_request_header("User-Agent", "Mozilla/5.0")
        txs.append(t)
    res = _parity(MULTI, gpuinspect.pack(txs))
    ai = list(gpuinspect.DEFAULT_EXPORTS).index("anomaly_score")
    scores = [int(v["tx_export"][ai]) for v in res.verdicts]
    assert scores[:2] == [1001, 1001]
    assert [int(v["status"]) for v in res.verdicts][:2] == [0, 0]
    assert scores[7] == 2002 and int(res.verdicts[7]["status"]) == 403
    batch = traffic.TrafficGen(traffic.SEED + 9).batch(800, attack_rate=0.3)
    _parity(MULTI, batch)


def test_gpu_tally_detail():
    """Detail tally (gi_tally_detail_get): the per-rule match counts equal the
    matched-rule lists counted on the host, the score histogram equals the
    summed per-PL inbound scores binned on the host (SURVEY §8(e) tally)."""
    text = open(CRS).read()
    batch = traffic.TrafficGen(traffic.SEED + 11).batch(3000, post_frac=0.2, attack_rate=0.3)
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    res = eng.inspect(batch)
    d = eng.tally_detail()
    assert len(d["rule_ids"]) == len(d["rule_hits"]) == eng.tally_rule_count()
    assert d["rule_ids"] == sorted(set(d["rule_ids"]))
    want = {}
    for i in range(batch.n_req):
        for rid in res.matched_rules(i):
            want[rid] = want.get(rid, 0) + 1
    got = {rid: h for rid, h in zip(d["rule_ids"], d["rule_hits"]) if h}
    assert got == want
    b = [gpuinspect.score_hist_value(res.verdicts["tx_export"][i], rs.exports) for i in range(batch.n_req)]
    assert d["score_hist"] == [b.count(k) for k in range(64)]
    assert sum(1 for x in d["score_hist"] if x) > 1  # the histogram carries information
    assert sum(want.values()) == int(eng.tally()["matched_total"])


MATCHED = """SecRuleEngine On
SecRule ARGS "@rx (?i)select" "id:1,phase:2,pass,chain,t:none,t:urlDecodeUni"
    SecRule MATCHED_VARS "@rx (?i)from" "setvar:tx.anomaly_score=+5"
SecRule ARGS_NAMES "@rx ^q" "id:2,phase:2,pass,chain"
    SecRule MATCHED_VAR "@contains x" "chain"
    SecRule MATCHED_VAR_NAME "@streq ARGS_NAMES:qx" "setvar:tx.anomaly_score=+100"
SecRule REQUEST_HEADERS:User-Agent|ARGS "@rx bot" "id:3,phase:2,pass,t:lowercase,setvar:'tx.ua=%{MATCHED_VAR}',setvar:'tx.uan=%{MATCHED_VAR_NAME}'"
SecRule TX:UA "@rx crawler" "id:4,phase:2,pass,setvar:tx.anomaly_score=+10"
SecRule MATCHED_VARS_NAMES "@rx ua" "id:5,phase:2,pass,setvar:tx.anomaly_score=+1000"
SecRule MATCHED_VAR_NAME "@rx ^TX:ua$" "id:6,phase:2,pass,setvar:tx.anomaly_score=+20000"
SecRule &MATCHED_VARS "@eq 0" "id:7,phase:2,pass,setvar:tx.anomaly_score=+300000"
SecRule ARGS "@rx a" "id:8,phase:2,pass,chain"
    SecRule &MATCHED_VARS "@gt 1" "setvar:tx.anomaly_score=+4000000"
SecRule TX:UAN "@streq REQUEST_HEADERS:User-Agent" "id:10,phase:2,pass,setvar:tx.anomaly_score=+50000000"
SecRule TX:ANOMALY_SCORE "@ge 50000000" "id:9,phase:2,deny,status:403"
"""


def test_gpu_parity_matched_vars():
    """MATCHED_VAR / MATCHED_VAR_NAME / MATCHED_VARS / MATCHED_VARS_NAMES as
    targets (chains, counts) and macros (coraza transaction.go matchVariable;
    MATCHED_VARS reset before every rule): GPU vs oracle, the score pins the
    rule-by-rule outcome."""
    txs = []
    for q, ua in ((b"q=1+SELECT+x+FROM+t", b"Mozilla"), (b"qx=axb&b=select+1", b"GoodBot Crawler"),
                  (b"a=aa&b=ab", b"curl"), (b"qy=1&z=xyz", b"bot"), (b"x=Bot&q=select%20from", b"Mozilla")):
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?" + q)
        t.add_request_header("Host", "x")
        t.add_request_header("User-Agent", ua)
        txs.append(t)
    res = _parity(MATCHED, gpuinspect.pack(txs))
    ai = list(gpuinspect.DEFAULT_EXPORTS).index("anomaly_score")
    scores = [int(v["tx_export"][ai]) for v in res.verdicts]
    assert scores[0] % 10 == 5 and scores[1] // 50000000 == 1  # MATCHED_VARS chain; User-Agent name macro
    batch = traffic.TrafficGen(traffic.SEED + 13).batch(600, attack_rate=0.3)
    _parity(MATCHED, batch)


CAPTURE_RULES = r"""SecRuleEngine On
SecRequestBodyAccess On
SecAction "id:900,phase:1,pass,nolog,setvar:tx.allowed='|application/x-www-form-urlencoded| |multipart/form-data| |application/json|',setvar:tx.charsets='|utf-8| |iso-8859-1|'"
SecRule REQUEST_HEADERS:Content-Type "@rx ^[^;\s]+" "id:920420,phase:1,pass,capture,t:none,setvar:'tx.content_type=|%{tx.0}|',chain"
    SecRule TX:content_type "!@within %{tx.allowed}" "t:lowercase,setvar:tx.score=+5"
SecRule REQUEST_HEADERS:Content-Type "@rx charset\s*=\s*[\"']?([^;\"'\s]+)" "id:920480,phase:1,pass,capture,t:none,chain"
    SecRule TX:1 "!@within %{tx.charsets}" "t:lowercase,setvar:tx.score=+5"
SecRule ARGS "@rx (?i)(union|select)\s+(\w+)" "id:942,phase:2,pass,capture,t:urlDecodeUni,setvar:'tx.last=%{tx.2}',setvar:tx.score=+3"
SecRule ARGS_NAMES "!@rx ^([a-z]+)$" "id:943,phase:2,pass,capture,setvar:'tx.bad=%{tx.0}%{tx.1}'"
SecRule TX:SCORE "@ge 8" "id:949,phase:2,deny,status:403"
"""


def test_gpu_capture_parity():
    """Observable captures: the 920420 / 920480 chains read
    their parent's TX.0 / TX.1, 942 and 943 read their own groups in setvar
    (943 negated: captures from the names that do not make it match); the
    capture records (rule, group, bytes) are compared with the oracle's."""
    rs = gpuinspect.Ruleset(CAPTURE_RULES, tx_exports=["score", "content_type", "last", "bad"])
    assert rs.capture_rules == frozenset({920420, 920480, 942, 943})
    cts = [b"application/json; charset=utf-8", b"text/xml;charset=UTF-16", b"multipart/form-data; boundary=x",
           b"application/x-www-form-urlencoded", b"text/plain; charset = 'latin1'", b";charset=", b"",
           b"APPLICATION/JSON", b"x/y; charset=\"utf-8\"; a=b"]
    txs = []
    gen = traffic.TrafficGen(traffic.SEED + 7).batch(400, attack_rate=0.3)
    for i in range(gen.n_req):
        t = gen.request(i)
        t.headers = [(k, v) for k, v in t.headers if k.lower() != b"content-type"]
        if i % 3:
            t.add_request_header("Content-Type", cts[i % len(cts)])
        if i % 5 == 0:
            t.uri += b"&q=Union+Select+pass%20word&Q1=x"
        txs.append(t)
    batch = gpuinspect.pack(txs)
    eng = gpuinspect.Engine(rs, matched_cap=64, capture_cap=16, capture_bytes_cap=1024)
    res = eng.inspect(batch)
    cfg = coraza.parse_seclang(CAPTURE_RULES)
    orc = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    ncap = int(res.verdicts["capture_cnt"].sum())
    assert ncap > 300, ncap
    assert any(res.captures(i) and res.captures(i)[0][0] == 942 for i in range(batch.n_req))


def test_gpu_capture_pool_chunked(monkeypatch):
    """The capture areas live in one chunk-sized pool (runtime.cpp
    chunk_cap_bytes): a 64 KB budget cuts the batch into many request chunks
    that reuse it; verdicts, exports and capture records stay the oracle's."""
    monkeypatch.setenv("GI_CHUNK_CAP_BYTES", "65536")
    rs = gpuinspect.Ruleset(CAPTURE_RULES, tx_exports=["score", "content_type", "last", "bad"])
    txs = []
    gen = traffic.TrafficGen(traffic.SEED + 9).batch(600, attack_rate=0.3)
    for i in range(gen.n_req):
        t = gen.request(i)
        t.headers = [(k, v) for k, v in t.headers if k.lower() != b"content-type"]
        t.add_request_header("Content-Type", b"application/json; charset=utf-8" if i % 2 else b"text/xml;charset=x")
        if i % 4 == 0:
            t.uri += b"&q=Union+Select+pass%20word"
        txs.append(t)
    batch = gpuinspect.pack(txs)
    eng = gpuinspect.Engine(rs, matched_cap=64, capture_cap=16, capture_bytes_cap=1024)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(CAPTURE_RULES), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    assert int(res.verdicts["capture_cnt"].sum()) > 600


XML_RULES = r"""SecRuleEngine On
SecRequestBodyAccess On
SecRule REQUEST_HEADERS:Content-Type "^(?:application(?:/soap\+|/)|text/)xml" "id:200000,phase:1,t:none,t:lowercase,pass,nolog,ctl:requestBodyProcessor=XML"
SecRule REQBODY_ERROR "!@eq 0" "id:200002,phase:2,t:none,deny,status:400,msg:'%{reqbody_error_msg}'"
SecRule XML:/* "@rx (?i)(union\s+select|<script)" "id:942,phase:2,pass,t:none,t:urlDecodeUni,setvar:tx.score=+5"
SecRule XML://@* "@rx ^javascript:" "id:941,phase:2,pass,t:none,t:lowercase,setvar:tx.score=+5"
SecRule XML "@contains evilmonkey" "id:3001,phase:2,pass,setvar:tx.score=+1"
SecRule &XML:/* "@gt 3" "id:3002,phase:2,pass,setvar:tx.many=1"
SecRule XML:/* "@detectSQLi" "id:942100,phase:2,pass,setvar:tx.score=+2"
SecRule TX:SCORE "@ge 5" "id:949,phase:2,deny,status:403"
"""

XML_BODIES = [
    b'<a href="x&amp;y" b=\'2\' disabled>hello <b>wor&lt;ld</b>  </a>',
    b'<?xml version="1.0" encoding="UTF-8"?><r><![CDATA[ union select 1 ]]>t&#65;&#x42;&nbsp;&foo;</r>',
    b'plain text evilmonkey', b'<a>unclosed', b'<a></b>', b'<x><a></b></x>', b'<br>text<p>x</p><img src="javascript:alert(1)">',
    b'<?xml version="1.0" encoding="ISO-8859-1"?><a/>', b'<a b=c-d:e>&#0;</a>', b'1 < 2', b'<a>\r\nx\ry\r</a>',
    b'<!DOCTYPE x [<!ENTITY e "v">]><x a="1">t</x>', b'<a><!-- c -- d --></a>', b'<p:a xmlns:p="u">t</p:a>',
    b'<p:a></q:a>', b'\xef\xbb\xbf<a>x</a>', b'<a>\xff</a>', b'<q>1 UNION SELECT password FROM users</q>',
    b'<a>&lt;script&gt;alert(1)&lt;/script&gt;</a>', b'<r><i>1</i><i>2</i><i>3</i><i>4</i><i>5</i></r>',
    b'<a x="1\n2" y="&quot;z&quot;"/><b>\xc3\xa9t\xc3\xa9</b>', b'', b'<a>\n\t \xc2\xa0</a>', b'<![CDATA[x', b'<?xml version="2.0"?><a/>',
    b'<a>t]]>u</a>', b'<a b="<">', b'<a =b>', b'<a:b:c/>', b'<a>&#xD800;&#x110000;&#65</a>',
]


def test_gpu_xml_body_parity():
    """XML body processor (base rule 200000 -> ctl:requestBodyProcessor=XML):
    XML:/* and XML://@* values and the decoder's errors (REQBODY_ERROR ->
    200002 -> 400), against oracle/xmlbody.py."""
    txs = []
    for i, body in enumerate(XML_BODIES * 4):
        t = gpuinspect.Transaction(method=b"POST", uri=b"/api?i=%d" % i)
        t.add_request_header("Host", "x")
        t.add_request_header("Content-Type", ["application/xml", "text/xml; charset=utf-8", "application/soap+xml",
                                              "text/plain"][i % 4])
        t.write_request_body(body)
        txs.append(t)
    res = _parity(XML_RULES, gpuinspect.pack(txs))
    st = [res.interruption(i)["status"] if res.interruption(i) else 200 for i in range(len(txs))]
    assert 400 in st and 403 in st and 200 in st


BODY_LIMIT_RULES = """SecRuleEngine %s
SecRequestBodyAccess On
SecRequestBodyLimit 64
SecRequestBodyLimitAction %s
SecRule ARGS "@contains evil" "id:1,phase:2,pass,setvar:tx.score=+5"
SecRule INBOUND_DATA_ERROR "@eq 1" "id:2,phase:2,pass,setvar:tx.limit=1"
SecRule ARGS_COMBINED_SIZE "@gt 40" "id:3,phase:2,pass,setvar:tx.big=1"
SecRule REQUEST_HEADERS:X "@rx ." "id:4,phase:1,pass,setvar:tx.p1=1"
SecRule TX:SCORE "@ge 5" "id:9,phase:2,deny,status:403"
"""


@pytest.mark.parametrize("engine,action", [("On", "Reject"), ("On", "ProcessPartial"), ("DetectionOnly", "Reject")])
def test_gpu_body_limit(engine, action):
    """SecRequestBodyLimit: Reject -> 413 (no rule id, phase 1 matches kept),
    ProcessPartial -> the first limit bytes, a body of exactly the limit, and
    INBOUND_DATA_ERROR / ARGS_COMBINED_SIZE."""
    text = BODY_LIMIT_RULES % (engine, action)
    txs = []
    for n in (0, 10, 63, 64, 65, 100, 500):
        for evil_at in (0, 60):
            body = bytearray(b"a=" + b"x" * max(0, n - 2))[:n]
            if n >= evil_at + 7:
                body[evil_at:evil_at + 7] = b"&q=evil"
            t = gpuinspect.Transaction(method=b"POST", uri=b"/?g=1")
            t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
            t.add_request_header("X", "1")
            t.write_request_body(bytes(body))
            txs.append(t)
    rs = gpuinspect.Ruleset(text, tx_exports=["score", "limit", "big", "p1"])
    eng = gpuinspect.Engine(rs)
    batch = gpuinspect.pack(txs)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    if engine == "On" and action == "Reject":
        assert any(res.interruption(i) == {"rule_id": 0, "status": 413, "action": "deny", "phase": 2}
                   for i in range(len(txs)))


PARTIAL_PREFIX_RULES = """SecRuleEngine On
SecRequestBodyAccess On
SecRequestBodyLimit 64
SecRequestBodyLimitAction ProcessPartial
SecRule ARGS "@validateByteRange 32-126" "id:10,phase:2,pass,t:none,setvar:tx.bad=1"
SecRule ARGS_POST "@contains evil" "id:13,phase:2,pass,t:none,setvar:tx.evil=1"
SecRule REQUEST_HEADERS:X "@streq stop" "id:11,phase:2,deny,status:403"
SecRule ARGS "@rx mon[k]ey" "id:12,phase:2,deny,status:403,t:none"
"""


def test_gpu_gate_prefix_partial_body():
    """in the gate's first stage a RF2_PREFIX link's
    phase-A bits are trusted only when the body fields are the speculative
    parser's.  A ProcessPartial body over SecRequestBodyLimit is parsed by the
    interpreter (k_bparse skips it), so phase A never saw its fields: rule 10
    (@validateByteRange over ARGS) must still match it, and rule 11's
    interruption makes the first stage final (no bail to the body stage).
    A fresh engine runs its first batch with the gate on."""
    txs = []
    for n in (10, 40, 63, 64, 65, 100, 300):
        for stop in (False, True):
            for bad_at in (3, 50):
                body = bytearray(b"a=" + b"x" * max(0, n - 2))[:n]
                if n > bad_at + 3:
                    body[bad_at:bad_at + 3] = b"%01"
                if n > 30:
                    body[20:28] = b"&e=evil&"
                t = gpuinspect.Transaction(method=b"POST", uri=b"/?g=1")
                t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
                t.add_request_header("X", "stop" if stop else "go")
                t.write_request_body(bytes(body))
                txs.append(t)
    rs = gpuinspect.Ruleset(PARTIAL_PREFIX_RULES, tx_exports=["bad", "evil"])
    eng = gpuinspect.Engine(rs)
    batch = gpuinspect.pack(txs)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(PARTIAL_PREFIX_RULES), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    assert eng.stats()["gate_requests"] > 0, "the first batch of a context runs gated"
    # over-limit bodies with an out-of-range byte in the first 64 bytes, stopped by rule 11
    hit = [i for i in range(batch.n_req) if 10 in res.matched_rules(i) and 11 in res.matched_rules(i)]
    assert hit


def test_gpu_large_body_next_to_small():
    """One 24 MB body among small requests stages and runs (bounded k_long
    buffers: ADVICE r02) and every verdict matches the oracle."""
    text = ("SecRuleEngine On\nSecRequestBodyAccess On\nSecRequestBodyLimit 134217728\n"
            'SecRule ARGS|REQUEST_BODY "@rx evil[a-z]+monkey" "id:1,phase:2,deny,status:403,t:none,t:lowercase"\n')
    big = b"a=" + b"x" * (24 << 20) + b"&b=EVILbigMONKEY"
    txs = []
    for i in range(64):
        t = gpuinspect.Transaction(method=b"POST", uri=b"/?i=%d" % i)
        t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
        t.write_request_body(big if i == 5 else b"q=evilsmallmonkey" if i % 7 == 0 else b"q=ok")
        txs.append(t)
    res = _parity(text, gpuinspect.pack(txs))
    assert res.interruption(5) is not None and res.interruption(7) is not None and res.interruption(1) is None


@pytest.fixture
def engine_env(monkeypatch):
    """Engine tunables are read when a context is created (runtime.cpp gi_ctx_create)."""
    def set_env(**kv):
        for k, v in kv.items():
            monkeypatch.setenv(k, str(v))
    return set_env


def test_gpu_eval_wave_forced_crs_pl4(engine_env):
    """Every request through k_eval_wave (one wave per request: the 64-rule
    skip walk and the 64-field filters) on the PL4 ruleset and the C3 mix."""
    engine_env(GI_EVAL_WAVE_FIELDS=1)
    text = open(os.path.join(ROOT, "rulesets", "crs_pl4.conf")).read()
    batch = traffic.TrafficGen(traffic.SEED + 41).batch(300, post_frac=0.5, attack_rate=0.3)
    res = _parity(text, batch)
    assert int((res.verdicts["action"] != 0).sum()) > 30


def test_gpu_chunked_batch_crs_pl1(engine_env):
    """A tiny per-chunk queue-pool budget cuts the batch into many request
    chunks (gi_stage_batch), each a full pipeline pass: verdicts, matched ids
    and the batch tally stay those of one pass."""
    engine_env(GI_CHUNK_POOL_WORDS=3e5)
    text = open(CRS).read()
    batch = traffic.TrafficGen(traffic.SEED + 42).batch(400, post_frac=0.4, attack_rate=0.3)
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    eng.stage(batch)
    eng.run()
    eng.sync()
    res = eng.fetch()
    st = eng.stats()
    cfg = coraza.parse_seclang(text)
    orc = compare.oracle_verdicts(cfg, batch, rs.exports)
    assert not compare.compare(res, orc)
    t = eng.tally()
    assert t["n_req"] == batch.n_req
    assert t["matched_total"] == sum(len(v.matched) for v in orc.values())
    assert t["n_interrupted"] == sum(1 for v in orc.values() if v.rule_id or v.status)
    assert any(ln["name"] == "k_collect" for ln in st["launches"])


def _restricted_header_batch():
    """Requests for the CRS v4 920450 / 920451 shape (capture + setvar with a
    macro key + a chain over TX:/^header_name_9204xx_/ @within the restricted
    list) and the 921170 / 921180 parameter counters (PL3)."""
    names = ["Proxy", "Lock-Token", "Content-Range", "If", "Accept-Charset", "X-Http-Method-Override",
             "content-encoding", "PROXY", "If-None-Match", "Proxy-Connection", "X-Custom", "iF", "Ifx",
             # the phase-A name filter (compile.cpp within_chain_filters): names spanning list
             # entries, slashes, and names another TX key regex (921180's /paramcounter_.*/) can see
             "proxy/ /lock-token", "If/ /X-Http-Method", "/proxy", "proxy/", "X-Method-Override/ /x-middleware",
             "paramcounter_a", "X-Paramcounter_args:a", "ParamCounter_"]
    txs = []
    for i, n in enumerate(names):
        for extra in ([], [("Proxy", "b")], [(n, "again")], [("X-%d" % k, "v") for k in range(40)]):
            t = gpuinspect.Transaction(method=b"GET", uri=b"/p?a=1&b=%d" % i)
            t.add_request_header("Host", "example.com")
            t.add_request_header("User-Agent", "Mozilla/5.0")
            t.add_request_header(n, "value-%d" % i)
            for k, v in extra:
                t.add_request_header(k, v)
            txs.append(t)
    for uri in (b"/?a=1&a=2", b"/?a[]=1&a[]=2", b"/?a=1&b=2&A=3", b"/?x=1&x=2&x=3&y[]=1&y[]=2", b"/?q=evilmonkey"):
        for hn in (None, "paramcounter_x", "paramcounter_args:a"):
            t = gpuinspect.Transaction(method=b"GET", uri=uri)
            t.add_request_header("Host", "example.com")
            t.add_request_header("Accept", "*/*")
            if hn:
                t.add_request_header(hn, "1")
            txs.append(t)
    t = gpuinspect.Transaction(method=b"POST", uri=b"/form?a=1")
    t.add_request_header("Host", "example.com")
    t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
    t.write_request_body(b"a=2&b=3&b=4&c[]=1&c[]=2")
    txs.append(t)
    t = gpuinspect.Transaction(method=b"GET", uri=b"/")
    t.add_request_header("Host", "example.com")
    t.add_request_header("Pr\xc3\xb6xy", "non-ascii name")
    t.add_request_header("If", "x")
    txs.append(t)
    return gpuinspect.pack(txs)


@pytest.mark.parametrize("ruleset", ["crs_pl1", "crs_pl4"])
def test_gpu_macro_key_setvar_chains(ruleset):
    """setvar:'tx.header_name_920450_%{tx.0}=/%{tx.0}/' creates TX keys at run
    time; the chained TX:/^header_name_920450_/ reads them."""
    text = open(os.path.join(ROOT, "rulesets", ruleset + ".conf")).read()
    batch = _restricted_header_batch()
    res = _parity(text, batch)
    m = [res.matched_rules(i) for i in range(batch.n_req)]
    assert sum(920450 in x for x in m) >= 20      # Proxy, Lock-Token, Content-Range, If, ...
    assert sum(920450 not in x for x in m) >= 8   # Accept-Charset, X-Custom, If-None-Match, ...
    if ruleset == "crs_pl4":
        assert sum(920451 in x for x in m) >= 4   # Accept-Charset (PL2 extended list)
        assert sum(921180 in x for x in m) >= 2   # repeated parameter names (PL3)


def test_gpu_within_automaton():
    """@within over a literal / folded-constant argument runs the argument's
    suffix automaton on the device (compile.cpp within_dfa)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("tcb", os.path.join(ROOT, "tests", "test_cpu_baseline.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    text, batch = m.within_batch()
    res = _parity(text, batch)
    assert int((res.verdicts["status"] == 403).sum()) > 50


def test_gpu_uri_forms():
    """Absolute, scheme-relative, opaque, relative and invalid request-targets
    through the device's url.Parse / String restatement (k_collect), every
    URI variable compared through capture records."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("tcb", os.path.join(ROOT, "tests", "test_cpu_baseline.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    text, batch = m.uri_batch()
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, capture_cap=16, capture_bytes_cap=4096)
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc, max_report=100)
    assert not bad, bad
