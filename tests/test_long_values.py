"""Long values (>= GI_LONG_MIN = 2048 bytes) take k_long: one wave per
(item, stream), the chain run chunk-parallel and each admitted pattern
decided by its rule's own automaton (SURVEY §5 "long-context": no per-lane
transformation buffer, no transposed queue block).  GPU: the CRS-shaped PL1
ruleset (incl. libinjection) on long urlencoded / JSON / multipart values,
bit-exact with the oracle."""
import random

import pytest

import gpuinspect
from oracle import compare, coraza

CRS = "rulesets/crs_pl1.conf"
PAYLOADS = [b"<script>alert(1)</script>", b"1 UNION SELECT username FROM users", b"../../../../etc/passwd",
            b"admin' or 1=1--", b";cat /etc/passwd", b"javascript:alert(1)", b"<img src=x onerror=alert(1)>"]


def _filler(rng, n):
    alpha = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 -_.,%+&="
    return bytes(rng.choice(alpha) for _ in range(n))


def _requests(seed=7, n=48):
    rng = random.Random(seed)
    txs = []
    for i in range(n):
        size = rng.choice([2048, 3000, 9000, 40000])
        v = bytearray(_filler(rng, size))
        if i % 3 != 2:  # an attack somewhere inside the long value
            p = rng.choice(PAYLOADS)
            at = rng.randrange(0, len(v) - len(p))
            v[at:at + len(p)] = p
        v = bytes(v)
        kind = i % 3
        if kind == 0:
            q = b"".join(b"%%%02X" % c for c in v)
            t = gpuinspect.Transaction(method=b"POST", uri=b"/f")
            t.add_request_header(b"Host", b"localhost")
            t.add_request_header(b"Content-Type", b"application/x-www-form-urlencoded")
            t.write_request_body(b"short=1&long=" + q)
        elif kind == 1:
            t = gpuinspect.Transaction(method=b"POST", uri=b"/api")
            t.add_request_header(b"Host", b"localhost")
            t.add_request_header(b"Content-Type", b"application/json")
            s = v.replace(b"\\", b"").replace(b'"', b"")
            t.write_request_body(b'{"a": 1, "long": "' + s + b'"}')
        else:
            t = gpuinspect.Transaction(method=b"POST", uri=b"/up")
            t.add_request_header(b"Host", b"localhost")
            t.add_request_header(b"Content-Type", b"multipart/form-data; boundary=XyZ")
            t.write_request_body(b"--XyZ\r\nContent-Disposition: form-data; name=\"doc\"\r\n\r\n" + v +
                                 b"\r\n--XyZ--\r\n")
        txs.append(t)
    # a long value in a query argument and a header as well
    t = gpuinspect.Transaction(method=b"GET", uri=b"/?q=" + b"a" * 3000 + b"%3Cscript%3Ealert(1)%3C/script%3E")
    t.add_request_header(b"Host", b"localhost")
    t.add_request_header(b"User-Agent", b"x" * 2500 + b" union select 1 from t")
    txs.append(t)
    return txs


@pytest.mark.gpu
def test_gpu_long_values_parity():
    text = open(CRS).read()
    rs = gpuinspect.Ruleset(text)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    batch = gpuinspect.pack(_requests())
    res = eng.inspect(batch)
    orc = compare.oracle_verdicts(coraza.parse_seclang(text), batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    assert int((res.verdicts["action"] != 0).sum()) > 10
