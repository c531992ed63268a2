"""CPU-side checks of the product library (no GPU needed): the C-ABI loads
and exports every symbol include/gpuinspect.h declares, the SecLang compiler
accepts/rejects what the oracle accepts/rejects, and the @rx DFA compiler
agrees with the oracle's Go-regexp restatement on random inputs."""
import json
import os
import random
import re

import pytest

import gpuinspect
from oracle import coraza, goregex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def test_header_symbols_exported():
    lib = gpuinspect.load_library()
    hdr = open(os.path.join(ROOT, "include", "gpuinspect.h")).read()
    decl = set(re.findall(r"\b(gi_[a-z_0-9]+)\s*\(", hdr))
    assert decl, "no declarations parsed"
    assert decl == set(gpuinspect.EXPORTED_SYMBOLS), decl ^ set(gpuinspect.EXPORTED_SYMBOLS)
    for name in decl:
        assert hasattr(lib, name), name


def test_kat_rulesets_compile():
    kats = json.load(open(os.path.join(GOLDEN, "kats.json")))
    for sc in kats["scenarios"]:
        text = gpuinspect.aggregate_configmaps(sc["configmaps"])
        rs = gpuinspect.Ruleset(text)
        assert rs.info["n_rules"] >= 1


BAD = [
    ('SecRule ARGS "@rx (" "id:1,deny"', "parse"),
    ('SecRule ARGS "@rx a" "id:1,bogus"', "parse"),
    ('SecRule NOPE "@rx a" "id:1"', "parse"),
    ('SecRule ARGS "@rx a" "phase:2,deny"', "parse"),  # no id
    ('SecFoo bar', "parse"),
    ('SecRule ARGS "@rx a" "id:1,chain"', "parse"),   # unterminated chain
]


@pytest.mark.parametrize("text,kind", BAD)
def test_compile_rejects_like_oracle(text, kind):
    with pytest.raises(coraza.SecLangError):
        coraza.parse_seclang(text)
    with pytest.raises(gpuinspect.SecLangError) as e:
        gpuinspect.Ruleset(text)
    assert e.value.code == gpuinspect.GI_EPARSE


def test_unsupported_is_flagged_not_guessed():
    with pytest.raises(gpuinspect.SecLangError) as e:
        gpuinspect.Ruleset('SecRule ARGS "@verifyCC \\d{13,16}" "id:1,deny"')
    assert e.value.code == gpuinspect.GI_EUNSUPPORTED


PATTERNS = [
    r"(?i:(\b(select|union|insert|update|delete|drop)\b.*\b(from|into|where|table)\b))",
    r"(?i:<script[^>]*>.*?</script>|javascript:|onerror\s*=|onload\s*=|<iframe)",
    r"^(?:GET|HEAD)$", r"\bfoo\b", r"a.b", r"(?i)k", r"[^\x00-\x7f]", r"(?m)$\n^", r".{3}",
    r"(?:^|[\\/])\.\.(?:[\\/]|$)", r"\Aab|cd\z", r"(?i)[a-z]+s$", r"\d+\s*=\s*\d+", r"(a|b){2,4}c",
]


@pytest.mark.parametrize("pat", PATTERNS)
def test_regex_dfa_matches_oracle(pat):
    rnd = random.Random(hash(pat) & 0xFFFF)
    alpha = b"abcxzsSkK select from or = '\"\n<>/\\.-_0129\xc3\xa9\xe2\x84\xaa\xff\xc3\x41\xe1\x80"
    g = goregex.compile_go("(?sm)" + pat)
    for _ in range(800):
        s = bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 20)))
        rc, _ = gpuinspect.selftest_regex("(?sm)" + pat, s)
        assert rc in (0, 1)
        assert rc == int(g.match_string(s)), (pat, s)


CAPTURE_LOGDATA = """SecRuleEngine On
SecRule ARGS "@rx (?i)(union)\\s+(select)" "id:1,phase:2,pass,capture,t:none,t:urlDecodeUni,\\
    logdata:'Matched Data: %{TX.0} found within %{MATCHED_VAR_NAME}',setvar:'tx.score=+5'"
SecRule TX:SCORE "@ge 5" "id:2,phase:2,deny,status:403"
"""


def test_capture_without_reader_compiles():
    """capture whose TX.0-TX.9 only feed logdata (the CRS pattern) is exact to drop."""
    rs = gpuinspect.Ruleset(CAPTURE_LOGDATA)
    assert rs.info["n_rules"] == 2


CAPTURE_READ = [
    # a chained link reads the captured value (CRS 920420 / 920480 style): fed in chain
    ('SecRule REQUEST_HEADERS:Content-Type "@rx ^([^;]+)" "id:1,phase:1,deny,capture,chain"\n'
     'SecRule TX:1 "!@within text/plain" ""', False),
    # the capturing rule's own setvar reads it (its captures precede its actions)
    ('SecRule ARGS "@rx (a+)" "id:1,phase:2,pass,capture,setvar:tx.seen=%{tx.1}"', False),
    # a later rule reads it: every capture of the program is observable
    ('SecRule ARGS "@rx (a+)" "id:1,phase:2,pass,capture"\nSecRule ARGS "@streq %{TX.0}" "id:2,phase:2,deny"', True),
    # whole-collection / regex-keyed / counted TX targets can see TX.0
    ('SecRule ARGS "@rx (a+)" "id:1,phase:2,pass,capture"\nSecRule TX "@rx aa" "id:2,phase:2,deny"', True),
    ('SecRule ARGS "@rx (a+)" "id:1,phase:2,pass,capture"\nSecRule TX:/^[0-9]$/ "@rx aa" "id:2,phase:2,deny"', True),
    ('SecRule ARGS "@rx (a+)" "id:1,phase:2,pass,capture"\nSecRule &TX:0 "@eq 1" "id:2,phase:2,deny"', True),
]


@pytest.mark.parametrize("text,glob", CAPTURE_READ)
def test_capture_with_reader_compiles(text, glob):
    """Observable captures compile to a device submatch program (pike.h); the
    plan lists the rules whose captures are recorded."""
    coraza.parse_seclang(text)  # valid SecLang
    rs = gpuinspect.Ruleset(text)
    assert 1 in rs.capture_rules


def test_capture_analysis_keeps_logdata_captures_dropped():
    """A 920420-style chain makes only its own capture observable: the CRS
    detection rules' logdata captures stay dropped."""
    text = (CAPTURE_LOGDATA + 'SecRule REQUEST_HEADERS:Content-Type "@rx ^[^;\\s]+" '
            '"id:920420,phase:1,pass,capture,setvar:\'tx.ct=|%{tx.0}|\',chain"\n'
            'SecRule TX:ct "!@within |text/plain|" "setvar:tx.score=+5"\n')
    rs = gpuinspect.Ruleset(text)
    assert rs.capture_rules == frozenset({920420})
    # with a reader outside any chain every capture is observable
    rs2 = gpuinspect.Ruleset(text + 'SecRule TX:0 "@rx x" "id:9,phase:2,pass"\n')
    assert rs2.capture_rules == frozenset({1, 920420})


def test_capture_observable_on_pm_is_unsupported():
    text = 'SecRule ARGS "@pm foo bar" "id:1,phase:2,pass,capture"\nSecRule TX:0 "@rx foo" "id:2,phase:2,deny"'
    coraza.parse_seclang(text)
    with pytest.raises(gpuinspect.SecLangError) as e:
        gpuinspect.Ruleset(text)
    assert e.value.code == gpuinspect.GI_EUNSUPPORTED


def test_capture_exported_compiles():
    rs = gpuinspect.Ruleset(CAPTURE_LOGDATA, tx_exports=["score", "0"])
    assert rs.capture_rules == frozenset({1})


CAPTURE_PATTERNS = [
    r"^[^;\s]+", r"charset\s*=\s*[\"']?([^;\"'\s]+)", r"(a+?)(b*)", r"(a|ab)(c|bcd)(d*)", r"((a)|b)+",
    r"(?i)(k)(s)?", r"\b(\w+)\b", r"^(.*)$", r"(x)?(y)?z", r"(a{2,3})(a*)", r"(?:(\d+)-)+(\d+)",
    r"(?i:(select|union)\s+(all\s+)?(\w+))", r"(<)(script|img)([^>]*)(>?)", r"([^\x00-\x7f]+)(.)",
    r"(a*?)(a*?)b", r"(.)(.)(.)(.)(.)(.)(.)(.)(.)(.)(.)", r"(?m)^(ab|cd)$",
]


@pytest.mark.parametrize("pat", CAPTURE_PATTERNS)
def test_capture_vm_matches_oracle(pat):
    """The submatch VM k_eval runs (pike.h, here on the host) against the
    oracle's FindStringSubmatch restatement on random strings: the match and
    every group 0..8."""
    rnd = random.Random(hash(pat) & 0xFFFF)
    alpha = b"aabbcdxyzkKsS select union all 09-<>script img\n;='\"\xc3\xa9\xe2\x84\xaa\xff"
    g = goregex.compile_go("(?sm)" + pat)
    for _ in range(400):
        s = bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 24)))
        got = gpuinspect.selftest_capture(pat, s)
        exp = g.find_string_submatch(s)
        if exp is None:
            assert got is None, (pat, s, got)
            continue
        assert got is not None, (pat, s, exp)
        vals = [s[a:b] if x else b"" for x in got for a, b in [x or (0, 0)]]
        assert vals == exp[:9], (pat, s, vals, exp)


PMF_RULES = """SecRuleEngine On
SecRule ARGS|REQUEST_HEADERS:User-Agent "@pmFromFile scanners.data" "id:10,phase:2,deny,status:403,t:none,t:lowercase"
SecRule ARGS "!@pmFromFile allow.data" "id:11,phase:2,pass"
"""
PMF_FILES = {
    "scanners.data": b"# scanner user agents\r\nNikto\r\n  sqlmap  \n\n#comment\nunion select\nEvil Monkey",
    "allow.data": b"ok\nfine\n",
}


def test_pm_file_phrases_restatement():
    assert coraza.pm_file_phrases(PMF_FILES["scanners.data"]) == [
        b"nikto", b"sqlmap", b"union select", b"evil monkey"]
    assert coraza.pm_file_phrases(b"") == []


def test_pmfromfile_compiles_with_data_files():
    coraza.parse_seclang(PMF_RULES, PMF_FILES)
    rs = gpuinspect.Ruleset(PMF_RULES, data_files=PMF_FILES)
    assert rs.info["n_rules"] == 2 and rs.info["n_hit_slots"] == 2  # both links are phase-A scanned


def test_pmfromfile_missing_file_is_a_parse_error():
    with pytest.raises(coraza.SecLangError):
        coraza.parse_seclang(PMF_RULES, {"scanners.data": b"x"})
    with pytest.raises(gpuinspect.SecLangError) as e:
        gpuinspect.Ruleset(PMF_RULES, data_files={"scanners.data": b"x"})
    assert e.value.code == gpuinspect.GI_EPARSE
    assert "allow.data" in str(e.value)


def test_multimatch_links_scan_prefix_streams():
    # multiMatch links are phase-A scanned on every prefix of their chain (one
    # stream per prefix, one slot); with a residual target (REQUEST_BODY) they
    # stay interpreter-only (the clear-bit path tests final values only)
    text = ('SecRule ARGS "@rx ^abc$" "id:1,phase:2,pass,multiMatch,t:lowercase,t:trim"\n'
            'SecRule ARGS "@rx ^abc$" "id:2,phase:2,pass,t:lowercase"\n'
            'SecRule ARGS|REQUEST_BODY "@rx ^abc$" "id:3,phase:2,pass,multiMatch,t:lowercase"')
    coraza.parse_seclang(text)
    rs = gpuinspect.Ruleset(text)
    assert rs.info["n_rules"] == 3 and rs.info["n_hit_slots"] == 2
    assert rs.info["n_scan_streams"] >= 3  # (), (lowercase), (lowercase, trim)


# Flag groups persist across '|' to the end of the enclosing group (Go
# regexp/syntax); CRS 941xxx relies on it: "(?i)<(?:script..)\b|\bon[a-z]{3,25}=".
FLAG_SCOPE = [r"a(?i)b|c", r"(?:(?i)a)|b", r"x|(?i)y|z", r"(?i)<script\b|\bon[a-z]{3,25}[\s\x0b]*=|javascript:",
              r"(?:a(?i)b|c)d", r"(?s-i:A)|(?i)b"]


@pytest.mark.parametrize("pat", FLAG_SCOPE)
def test_regex_flag_scope_matches_oracle(pat):
    rnd = random.Random(len(pat))
    alpha = b"abcdABCDxyzXYZ <scriptSCRIPT onON=:\xc5\xbf\xe2\x84\xaa"
    g = goregex.compile_go("(?sm)" + pat)
    strs = [b"C", b"aB", b"B", b"Z", b".oNuvw=", b"a.ONUVW=", b"Cd", b"A", b"a"] + [
        bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 16))) for _ in range(400)]
    got, _ = gpuinspect.selftest_regex_many("(?sm)" + pat, strs)
    for s, rc in zip(strs, got):
        assert rc == int(g.match_string(s)), (pat, s)


# Unbounded counted repetition x{m,} (= x{m-1} x+): found by the bench's
# parity sample (CRS 941101's relaxed phase-A automaton required m+1 copies).
UNBOUNDED = [r"a{2,}", r"^a{3,}$", r"x(?:ab){2,}y", r"[a-c]{4,}", r"a{1,}", r"a{0,}b", r"(?i)\bon[a-z]{3,}[\s\x0b]*="]


@pytest.mark.parametrize("pat", UNBOUNDED)
def test_unbounded_repeat_matches_oracle(pat):
    rnd = random.Random(len(pat) * 3)
    alpha = b"abcxyON= "
    g = goregex.compile_go("(?sm)" + pat)
    strs = [b"aa", b"aaa", b"aaaa", b"xababy", b"xaby", b"abca", b"abc", b".oNuvw=", b"onab="] + [
        bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 12))) for _ in range(600)]
    got, n_states = gpuinspect.selftest_regex_many("(?sm)" + pat, strs)
    assert n_states > 0  # the DFA path
    for s, rc in zip(strs, got):
        assert rc == int(g.match_string(s)), (pat, s)


# Patterns whose search DFA exceeds the state cap: the exact matcher is the
# NFA position tables (host walk == the device's nfa_match), the phase-A
# automaton a superset relaxation.
EXPLODING = [r"(?i)<(?:script|iframe|object|svg|style|link)\b|\bon[a-z]{3,25}[\s\x0b]*=|javascript[\s\x0b]*:",
             r"(?i)on[a-z]{3,25}=", r"[ab]*a[ab]{16}c", r"(?:x|\bq)[a-z]{2,30}\b!(?i)on[a-z]{3,25}"]


@pytest.mark.parametrize("pat", EXPLODING)
def test_nfa_fallback_matches_oracle(pat):
    rnd = random.Random(len(pat) * 7)
    alpha = b"abcnoqxONQ=!c \t.\xc5\xbf\xe2\x84\xaa\xff"
    g = goregex.compile_go("(?sm)" + pat)
    strs = [b".oNuvw=", b"onabc=", b"\xc5\xbfonabc=", b"a" * 18 + b"c", b"x" + b"a" * 40 + b"!onabc"] + [
        bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 40))) for _ in range(800)]
    got, n_states = gpuinspect.selftest_regex_many("(?sm)" + pat, strs)
    assert n_states == 0  # took the NFA path
    for s, rc in zip(strs, got):
        assert rc == int(g.match_string(s)), (pat, s)


def _crs_rx_patterns():
    import re as _re
    text = open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read()
    return sorted(set(_re.findall(r'"@rx ((?:[^"\\]|\\.)*)"', text)))


def test_crs_rx_patterns_match_oracle():
    """Every @rx of the CRS-shaped ruleset: host automaton (DFA, or the NFA
    tables where the DFA exceeds the cap) vs the oracle's Go-regexp
    restatement, on attack payloads, case variants and random strings."""
    import traffic
    pats = _crs_rx_patterns()
    assert len(pats) > 50
    rnd = random.Random(5)
    corpus = list(traffic.ATTACKS) + [a.upper() for a in traffic.ATTACKS] + [
        b".oNuvw=", b"x OnLoad =", b"JaVaScRiPt:", b"../../etc/passwd", b"\xc5\xbfonabc=", b"\xe2\x84\xaaey"]
    alpha = b"abcdefghijklmnopqrstuvwxyz ABCXYZ0123456789<>/\\'\";:=()[]{}.,-_|&$%*+!?#@\n\t\xc3\xa9"
    corpus += [bytes(rnd.choice(alpha) for _ in range(rnd.randint(0, 48))) for _ in range(60)]
    for pat in pats:
        p = pat.replace('\\"', '"')
        g = goregex.compile_go("(?sm)" + p)
        got, _ = gpuinspect.selftest_regex_many("(?sm)" + p, corpus)
        for s, rc in zip(corpus, got):
            assert rc == int(g.match_string(s)), (p, s)
