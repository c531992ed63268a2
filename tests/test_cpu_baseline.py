"""The CPU baseline (gi_cpu_baseline_inspect): the engine's own
interpreter compiled for the host, every rule link evaluated without phase A.

It is not the product path (gi_inspect_* only runs on the GPU) but it runs the
same interpreter source, so on CPU it also checks the interpreter-level
features against the oracle: compile-time folding (snapshot TX, folded runs,
constant links), macro-key setvar chains, body processors, libinjection.
"""
import os

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _check(text, batch, threads=4):
    rs = gpuinspect.Ruleset(text)
    res, secs = gpuinspect.cpu_baseline_inspect(rs, batch, threads=threads, matched_cap=128)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    assert secs > 0
    return res


CASES = [
    ("samples", os.path.join(GOLDEN, "samples_ruleset.conf"), 600, dict(attack_rate=0.3)),
    ("crs_pl1_get", os.path.join(ROOT, "rulesets", "crs_pl1.conf"), 400, dict(attack_rate=0.3)),
    ("crs_pl1_post", os.path.join(ROOT, "rulesets", "crs_pl1.conf"), 60, dict(attack_rate=0.3, post_frac=0.5)),
    ("crs_pl4_mix", os.path.join(ROOT, "rulesets", "crs_pl4.conf"), 120, dict(attack_rate=0.3, post_frac=0.5)),
    ("crs_ftw", os.path.join(ROOT, "rulesets", "crs_ftw.conf"), 150, dict(attack_rate=0.5)),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_cpu_baseline_matches_oracle(case):
    _, path, n, kw = case
    batch = traffic.TrafficGen(traffic.SEED + 11).batch(n, **kw)
    res = _check(open(path).read(), batch)
    assert int(res.verdicts["match_cnt"].astype(bool).sum()) > 0


@pytest.mark.parametrize("ruleset", ["crs_pl1", "crs_pl4"])
def test_cpu_baseline_macro_key_chains(ruleset):
    """CRS v4 920450 / 920451 (capture + setvar:'tx.header_name_9204xx_%{tx.0}=...'
    + TX:/^header_name_9204xx_/ chain) and 921170 / 921180 (paramcounter)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("tgp", os.path.join(ROOT, "tests", "test_gpu_parity.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    batch = m._restricted_header_batch()
    res = _check(open(os.path.join(ROOT, "rulesets", ruleset + ".conf")).read(), batch)
    ids = [res.matched_rules(i) for i in range(batch.n_req)]
    assert sum(920450 in x for x in ids) >= 20
    if ruleset == "crs_pl4":
        assert sum(920451 in x for x in ids) >= 4 and sum(921180 in x for x in ids) >= 2


def test_cpu_baseline_kats():
    import json
    kats = json.load(open(os.path.join(GOLDEN, "kats.json")))
    for sc in kats["scenarios"]:
        rs = gpuinspect.Ruleset(gpuinspect.aggregate_configmaps(sc["configmaps"]))
        txs = []
        for r in sc["requests"]:
            t = gpuinspect.Transaction()
            t.process_uri(r["uri"], r["method"], r["proto"])
            for k, v in r["headers"]:
                t.add_request_header(k, v)
            t.write_request_body(r["body"])
            txs.append(t)
        res, _ = gpuinspect.cpu_baseline_inspect(rs, txs, threads=2)
        for i, r in enumerate(sc["requests"]):
            it = res.interruption(i)
            assert (it["status"] if it else 200) == r["expect_status"], (sc["name"], r["uri"])


def test_cpu_baseline_threads_agree():
    text = open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read()
    rs = gpuinspect.Ruleset(text)
    batch = traffic.TrafficGen(traffic.SEED + 12).batch(300, attack_rate=0.3)
    a, _ = gpuinspect.cpu_baseline_inspect(rs, batch, threads=1)
    b, _ = gpuinspect.cpu_baseline_inspect(rs, batch, threads=7)
    assert (a.verdicts == b.verdicts).all() and (a.matched == b.matched).all()


def within_batch():
    """@within over a constant argument (compile.cpp within_dfa: the argument's
    suffix automaton) -- substrings, near misses, bytes >= 0x80, empty."""
    import random
    import urllib.parse
    rnd = random.Random(1)
    arg = "/content-encoding/ /proxy/ /lock-token/ /content-range/ /if/ /x-http-method-override/ GET HEAD POST \x01\xff ab\xc3\xa9"
    vals = ["", "/proxy/", "/proxy", "proxy/ /", "GET", "get", "/if/ /x", "zz", "\x01\xff", "\xc3\xa9", arg, arg + "x", " "]
    vals += ["".join(rnd.choice(arg) for _ in range(rnd.randint(1, 6))) for _ in range(300)]
    vals += [arg[i:j] for i, j in (sorted(rnd.sample(range(len(arg) + 1), 2)) for _ in range(300))]
    txs = []
    for v in vals:
        t = gpuinspect.Transaction(method=b"GET", uri=b"/?a=" + urllib.parse.quote(v.encode("latin-1")).encode())
        t.add_request_header("Host", "x")
        txs.append(t)
    text = ('SecRuleEngine On\nSecAction "id:9,phase:1,pass,setvar:tx.list=%s"\n'
            'SecRule ARGS "@within %s" "id:1,phase:2,pass,setvar:tx.anomaly_score=+1"\n'
            'SecRule ARGS "@within %%{tx.list}" "id:2,phase:2,deny,status:403"\n' % (arg[:40], arg))
    return text, gpuinspect.pack(txs)


def test_cpu_baseline_within_automaton():
    text, batch = within_batch()
    res = _check(text, batch)
    assert int((res.verdicts["status"] == 403).sum()) > 50


# request-target forms (Go net/url Parse + String, coraza ProcessURI): origin,
# absolute, scheme-relative, asterisk, opaque, relative, and Parse errors
URIS = [b"/", b"*", b"/a b?x=1", b"/%zz?q=1", b"/p%41th?a=%u0041", b"/x?", b"/x??a=1", b"/x#frag?q=1", b"//double?q=1",
        b"http://h/x", b"HTTP://H.example.com:8080/a/b?c=d", b"http://user:pa%20ss@h/p", b"http://us%2Fer@h/", b"http://a@b@c/",
        b"https://[::1]:443/x?y", b"http://[::1/x", b"http://[fe80::1]:8a/", b"http://h:80x/", b"http://h:/x", b"http://h%41/",
        b"http://h%C3%A9/x", b"http://h\xc3\xa9/x", b"http://h^/x", b"http://h/%zz", b"http://h", b"http://h?q=1", b"http:/x",
        b"http:x", b"mailto:a@b?subject=x", b"a:b", b"1a:b", b"a/b:c", b"a:b/c", b":x", b"relative/path?q=1",
        b"rel%20ative", b"./x:y", b"///triple", b"////q", b"//", b"//?q=1", b"//h", b"//@h/x", b"//u:@h/", b"http://h/a%2fb",
        b"http://h/caf\xc3\xa9", b"h+t-t.p://x/y", b"http://h/p?", b"http:///x", b"HtTp://h#f", b"/\x7f", b"http://u!$&'()*+,;=:~@h/",
        b"http://u%zz@h/", b"http://u\xc3@h/", b"?x=1", b"#x", b"", b"http://[::1]/p", b"http://[::1%25en0]/p", b"http://h/?a=1&b=2#c"]


def uri_batch():
    """Every URI-derived variable is captured (capture records are compared:
    REQUEST_URI, REQUEST_FILENAME, REQUEST_BASENAME, QUERY_STRING, ARGS, ARGS_NAMES)."""
    text = "SecRuleEngine On\n"
    for i, var in enumerate(["REQUEST_URI", "REQUEST_FILENAME", "REQUEST_BASENAME", "QUERY_STRING", "ARGS", "ARGS_NAMES"]):
        text += 'SecRule %s "@rx ^.*$" "id:%d,phase:1,pass,capture,setvar:tx.v%d=%%{tx.0}"\n' % (var, 10 + i, i)
    txs = []
    for u in URIS:
        t = gpuinspect.Transaction(method=b"GET", uri=u)
        t.add_request_header("Host", "x")
        txs.append(t)
    return text, gpuinspect.pack(txs)


def test_cpu_baseline_uri_forms():
    text, batch = uri_batch()
    rs = gpuinspect.Ruleset(text)
    res, _ = gpuinspect.cpu_baseline_inspect(rs, batch, threads=2, capture_cap=16, capture_bytes_cap=4096)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    assert not compare.compare(res, orc, max_report=100)
    # only the IPv6 zone form is outside the restatement
    assert [URIS[i] for i, v in orc.items() if v.unsupported] == [b"http://[::1%25en0]/p"]


def test_oracle_go_url_known_answers():
    """Go net/url String() / Path / RawQuery of forms whose results the Go
    documentation and net/url tests fix (url_test.go-style cases)."""
    cases = [
        (b"http://www.google.com/?q=go+language", b"http://www.google.com/?q=go+language", b"/", b"q=go+language"),
        (b"http://user:password@google.com", b"http://user:password@google.com", b"", b""),
        (b"mailto:webmaster@golang.org", b"mailto:webmaster@golang.org", b"", b""),
        (b"http://www.google.com/file%20one%26two", b"http://www.google.com/file%20one%26two", b"/file one&two", b""),
        (b"//foo", b"//foo", b"", b""),
        (b"http://[fe80::1]:8080/", b"http://[fe80::1]:8080/", b"/", b""),
        (b"http:%2f%2fwww.google.com/?q=go+language", b"http:%2f%2fwww.google.com/?q=go+language", b"", b"q=go+language"),
        (b"http://www.google.com/?", b"http://www.google.com/?", b"/", b""),
        (b"/foo?query=http://bad", b"/foo?query=http://bad", b"/foo", b"query=http://bad"),
    ]
    for raw, s, p, q in cases:
        v, _ = coraza.process_uri(raw)
        assert (v["REQUEST_URI"], v["REQUEST_FILENAME"], v["QUERY_STRING"]) == (s, p, q), raw
