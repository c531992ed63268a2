"""MULTIPART body processor (coraza internal/bodyprocessors/multipart.go over
Go's mime/multipart): FILES, FILES_NAMES, FILES_SIZES, FILES_COMBINED_SIZE,
MULTIPART_PART_HEADERS, ARGS_POST, MULTIPART_STRICT_ERROR / REQBODY_ERROR
(CRS base rules 200002 / 200003 deny with 400,
/root/reference/hack/generate_coreruleset_configmaps.py:73-89).

CPU: the oracle restatement (oracle/multipart.py) on hand-checked vectors of
Go's documented behaviour -- parity unpinned beyond them (no Go toolchain or
coraza source here).  GPU: kernels.hip parse_multipart (k_bparse and k_eval)
vs the oracle, bit-exact verdicts on edge cases and a seeded mix."""
import numpy as np
import pytest

import gpuinspect
from oracle import compare, coraza
from oracle import multipart as M

CT = b"multipart/form-data; boundary=AaB03x"
BASIC = (b"--AaB03x\r\nContent-Disposition: form-data; name=\"field1\"\r\n\r\nJoe Blow\r\n"
         b"--AaB03x\r\nContent-Disposition: form-data; name=\"pics\"; filename=\"file1.txt\"\r\n"
         b"Content-Type: text/plain\r\n\r\n... contents of file1.txt ...\r\n--AaB03x--\r\n")


def test_oracle_basic():
    r = M.process(BASIC, CT)
    assert r["error"] is None
    assert r["args_post"] == [(b"field1", b"Joe Blow")]
    assert r["files"] == [(b"", b"file1.txt")]
    assert r["files_names"] == [(b"", b"pics")]
    assert r["files_sizes"] == [(b"file1.txt", b"29")]
    assert r["combined_size"] == b"37"
    assert r["part_headers"] == [(b"field1", b'Content-Disposition: form-data; name="field1"'),
                                 (b"pics", b'Content-Disposition: form-data; name="pics"; filename="file1.txt"'),
                                 (b"pics", b"Content-Type: text/plain")]


@pytest.mark.parametrize("body,ct,err", [
    (BASIC.replace(b"\r\n", b"\n"), CT, None),                            # LF-only lines (first delimiter decides)
    (b"preamble\r\nmore\r\n" + BASIC + b"epilogue", CT, None),            # preamble / epilogue skipped
    (BASIC[:-12], CT, "unexpected EOF"),                                   # no closing delimiter: the part never ends
    (BASIC[:-2], CT, None),                                                # "--AaB03x--" at EOF without NL
    (BASIC, b"multipart/form-data", "multipart: boundary is empty"),
    (BASIC, b"multipart/form-data; boundary=a; boundary=b", "mime: invalid media type"),  # duplicate parameter
    (BASIC, b"text/plain; boundary=AaB03x", "not a multipart body"),
    (BASIC, b'multipart/form-data; boundary="AaB03x"', None),
    (b"--AaB03x\r\n Content-Disposition: form-data\r\n\r\nx\r\n--AaB03x--", CT,
     "multipart: NextPart: malformed MIME header"),                        # initial header line starts with space
    (b"--AaB03x\r\nBad Header: 1\r\n\r\nx\r\n--AaB03x--", CT, "multipart: NextPart: malformed MIME header"),
    (b"--AaB03x\r\nContent-Disposition: form-data; name=a\r\n\r\nx\r\n--AaB03x\r\nrubbish\r\n", CT,
     "multipart: NextPart: malformed MIME header"),                        # second part's header line without a colon
    (b"x" * 5000 + b"\r\n" + BASIC, CT, "multipart: NextPart: bufio: buffer full"),
    (b"--AaB03x\r\nContent-Disposition: form-data; name=a\r\n\r\nx\r\n--AaB03xNOT\r\n--AaB03x--", CT, None),
    (b"--AaB03x\r\nContent-Disposition: form-data; name=a\r\n\r\nx\r\njunk\r\n--AaB03x--", CT, None),
    (b"--AaB03x\r\nContent-Disposition: form-data; name=a\r\n\r\nx\r\n\r\njunk--AaB03x--", CT, "unexpected EOF"),
])
def test_oracle_edges(body, ct, err):
    assert M.process(body, ct)["error"] == err


def test_oracle_details():
    # continuation lines joined with one space; keys canonicalised; data "--AaB03xNOT" is data
    b = (b"--AaB03x\r\ncontent-disposition: form-data;\r\n\t name=\"a\"\r\nX-FOO-bar: 1\r\n\r\n"
         b"v\r\n--AaB03xNOT\r\n--AaB03x--")
    r = M.process(b, CT)
    assert r["args_post"] == [(b"a", b"v\r\n--AaB03xNOT")]
    assert r["part_headers"] == [(b"a", b'Content-Disposition: form-data; name="a"'), (b"a", b"X-Foo-Bar: 1")]
    # not form-data: no name; SetIndex of the same file name (case-insensitive)
    b = (b"--B\r\nContent-Disposition: attachment; name=\"n\"; filename=\"A.TXT\"\r\n\r\n12345\r\n"
         b"--B\r\nContent-Disposition: form-data; name=\"m\"; filename=\"a.txt\"\r\n\r\n12\r\n--B--")
    r = M.process(b, b"multipart/form-data; boundary=B")
    assert r["files"] == [(b"", b"A.TXT"), (b"", b"a.txt")]
    assert r["files_names"] == [(b"", b""), (b"", b"m")]
    assert r["files_sizes"] == [(b"A.TXT", b"2")]
    assert r["combined_size"] == b"7"
    with pytest.raises(M.MultipartUnsupported):
        M.process(b"--B\r\nContent-Transfer-Encoding: quoted-printable\r\n\r\n=41\r\n--B--", b"multipart/x; boundary=B")


RULES = """SecRuleEngine On
SecRequestBodyAccess On
SecRule FILES "@rx [.]php$" "id:301,phase:2,pass,t:none,t:lowercase,setvar:tx.anomaly_score=+1"
SecRule FILES_NAMES "@rx ^up" "id:302,phase:2,pass,setvar:tx.anomaly_score=+10"
SecRule FILES_SIZES "@gt 10" "id:303,phase:2,pass"
SecRule MULTIPART_PART_HEADERS "@rx (?i)content-type: text/x" "id:304,phase:2,pass"
SecRule ARGS_POST "@rx evil" "id:305,phase:2,pass,t:none,t:urlDecodeUni,setvar:tx.anomaly_score=+100"
SecRule ARGS_NAMES "@rx ^f" "id:306,phase:2,pass"
SecRule FILES_COMBINED_SIZE "@gt 100" "id:307,phase:2,pass"
SecRule REQBODY_ERROR_MSG "@contains buffer full" "id:308,phase:2,pass"
SecRule FILES:foo "@rx ." "id:309,phase:2,pass"
SecRule MULTIPART_PART_HEADERS:upfile "@rx disposition" "id:310,phase:2,pass,t:none,t:lowercase"
SecRule &FILES "@eq 2" "id:311,phase:2,pass"
SecRule REQUEST_BODY "@rx ." "id:312,phase:2,pass"
SecRule ARGS|FILES|FILES_NAMES "@rx wicked" "id:313,phase:2,pass"
SecRule &FILES_TMPNAMES "@eq 0" "id:314,phase:2,pass"
SecRule REQBODY_ERROR "!@eq 0" "id:200002,phase:2,t:none,deny,status:400"
SecRule MULTIPART_STRICT_ERROR "!@eq 0" "id:200003,phase:2,t:none,deny,status:400"
"""


def _part(rng, i, crlf):
    nl = b"\r\n" if crlf else b"\n"
    r = rng.random()
    hdr = []
    name = [b"f%d" % i, b"upfile", b"doc", b"evil", b""][int(rng.integers(0, 5))]
    words = [b"abc", b"wicked", b"evil", b"%41", b"+", b"-", b"\r\n", b"--", b"x" * 40, b"data"]
    data = b" ".join(words[int(w)] for w in rng.integers(0, len(words), int(rng.integers(0, 12))))
    if r < 0.45:
        fn = [b"a.php", b"b.PHP", b"c.txt", b"evil.jpg", b"x\\\"y.php"][int(rng.integers(0, 5))]
        hdr.append(b'Content-Disposition: form-data; name="%s"; filename="%s"' % (name, fn))
        hdr.append([b"Content-Type: text/x-php", b"Content-Type: image/jpeg", b"content-type:  text/plain "][
            int(rng.integers(0, 3))])
    elif r < 0.9:
        hdr.append(b'Content-Disposition: form-data; name="%s"' % name)
        if rng.random() < 0.3:
            hdr.append(b"X-Extra: a" + nl + b"\tcontinued")
    else:
        hdr.append(b"Content-Disposition: inline")
    return nl.join(hdr) + nl + nl + data


def mixes(n, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        crlf = rng.random() < 0.8
        nl = b"\r\n" if crlf else b"\n"
        b = b"bNd%d" % int(rng.integers(0, 1000))
        parts = [_part(rng, k, crlf) for k in range(int(rng.integers(0, 5)))]
        body = b"".join(b"--" + b + nl + p + nl for p in parts) + b"--" + b + b"--" + nl
        if rng.random() < 0.2:
            body = b"preamble" + nl + body + b"epilogue"
        k = rng.random()
        if k < 0.08:
            body = body[:int(rng.integers(0, len(body)))]          # truncated
        elif k < 0.12:
            body = body.replace(b"Content-Disposition", b"Content Disposition", 1)
        elif k < 0.14:
            body = b"z" * 4200 + nl + body
        ct = b"multipart/form-data; boundary=" + (b'"%s"' % b if rng.random() < 0.3 else b)
        if rng.random() < 0.05:
            ct = b"multipart/form-data"
        out.append((ct, body))
    return out


def batch_of(items):
    txs = []
    for ct, body in items:
        t = gpuinspect.Transaction(method=b"POST", uri=b"/upload?fx=1")
        t.add_request_header("Host", "x")
        t.add_request_header("Content-Type", ct)
        t.write_request_body(body)
        txs.append(t)
    return gpuinspect.pack(txs)


def test_compile_multipart_rules():
    gpuinspect.Ruleset(RULES)
    coraza.parse_seclang(RULES)


def test_oracle_multipart_verdicts():
    cfg = coraza.parse_seclang(RULES)
    items = [(CT, BASIC), (CT, BASIC[:-12])] + mixes(60)
    batch = batch_of(items)
    v = compare.oracle_verdicts(cfg, batch, gpuinspect.DEFAULT_EXPORTS)
    assert v[0].rule_id == 0 and 306 in v[0].matched
    assert (v[1].rule_id, v[1].status) == (200002, 400)


@pytest.mark.gpu
def test_gpu_multipart_parity():
    items = [(CT, BASIC), (CT, BASIC[:-12]), (CT, BASIC.replace(b"\r\n", b"\n")),
             (b"multipart/form-data", BASIC), (CT, b"x" * 5000 + b"\r\n" + BASIC)] + mixes(400)
    batch = batch_of(items)
    rs = gpuinspect.Ruleset(RULES)
    res = gpuinspect.Engine(rs).inspect(batch)
    cfg = coraza.parse_seclang(RULES)
    verdicts = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:5]
    fired = {}
    for v in verdicts.values():
        for m in v.matched + ([v.rule_id] if v.rule_id else []):
            fired[m] = fired.get(m, 0) + 1
    for rid in (301, 302, 303, 304, 305, 306, 307, 308, 310, 311, 313, 314, 200002):
        assert fired.get(rid, 0) > 0, (rid, fired)
    assert 309 not in fired and 312 not in fired


def many_parts(n, seed=12):
    """Bodies of 40-300 parts (k_mpparse splits them over the lanes:
    wave_multipart), file names repeated across the split (FILES_SIZES keeps
    one entry per name), some with an epilogue or a broken part late in the body."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        b = b"mAnY%d" % i
        parts = [_part(rng, k, True) for k in range(int(rng.integers(40, 300)))]
        if i % 4 == 1:  # one file name in many parts, in two cases
            parts += [b'Content-Disposition: form-data; name="u"; filename="%s"\r\n\r\nxyz' % fn
                      for fn in (b"dup.php", b"DUP.php", b"dup.php")]
        body = b"".join(b"--" + b + b"\r\n" + p + b"\r\n" for p in parts) + b"--" + b + b"--\r\n"
        if i % 5 == 2:
            body += b"epilogue --" + b + b"\r\nmore"
        if i % 7 == 3:
            body = body.replace(b"Content-Disposition", b"Content Disposition", 1 + int(rng.integers(0, 40)))
        if i % 11 == 5:
            body = body[:len(body) - int(rng.integers(1, 200))]
        out.append((b"multipart/form-data; boundary=" + b, body))
    return out


@pytest.mark.gpu
def test_gpu_multipart_many_parts_parity():
    batch = batch_of(many_parts(48))
    rs = gpuinspect.Ruleset(RULES)
    res = gpuinspect.Engine(rs).inspect(batch)
    verdicts = compare.oracle_verdicts(coraza.parse_seclang(RULES), batch, rs.exports)
    bad = compare.compare(res, verdicts)
    assert not bad, bad[:5]
