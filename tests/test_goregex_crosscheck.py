"""Cross-check of the oracle's Go-regexp restatement (oracle/goregex.py)
against CPython's `re` compiled from the RAW pattern text.

goregex.py parses RE2 syntax itself and emits an expanded, flag-free Python
pattern; a mistake in that parser / expansion would be shared by the oracle
and (if the product's C++ parser made the same mistake) hidden from every
GPU parity test.  Here each `@rx` argument of the stand-in rulesets
(`rulesets/crs_pl1.conf`, the 20 CRS-scale regexes of
`crs_pl1_rxstress.conf`, a sample of C5's generated rules) goes through a
minimal, independent Go -> Python translation and the two engines are
compared on a synthetic corpus (C2/C3 traffic fields, their urldecoded and
lowercased forms, the attack payloads, the rxstress hit / near-miss
payloads, C5 snippets).

Go / CPython differences handled explicitly (not by the oracle's code):
* `(?sm)`: Coraza's prefix (rx.go) -> re.S | re.M.
* `\\s` / `\\S`: Go's class is [\\t\\n\\f\\r ] (no \\v); rewritten outside
  classes, expanded to explicit ranges inside a class.
* `\\d \\w \\b`: ASCII in Go -> re.ASCII.
* `(?flags)` in mid-pattern: Go scopes it to the rest of the enclosing group
  (across later `|` alternatives); CPython 3.10 would apply it globally.
  Rewritten to `(?flags:...)` per alternative.
* `\\z` (Go end of text) -> `\\Z`.
* Case folding: Go's (?i) is Unicode simple folding (k ~ U+212A,
  s ~ U+017F); with re.ASCII CPython folds ASCII only.  The corpus is ASCII
  only, where the two agree -- non-ASCII inputs are EXCLUDED here (rune vs
  byte semantics are covered by the GPU-vs-oracle tests, parity unpinned).
Patterns using constructs without a faithful CPython form are SKIPPED and
counted: `\\p{..}`, `[[:class:]]`, `\\Q..\\E`, `\\x{..}`, `{,n}`, `(?<name>`,
`(?U)`, octal escapes / digits after a backslash.
"""
import os
import re
import sys
import urllib.parse
import warnings

import pytest

import traffic
from oracle import coraza, goregex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_rxstress  # noqa: E402

_UNSUPPORTED = re.compile(r"\\[pPQC]|\\x\{|\[\[:|\{,|\(\?<[A-Za-z]|\(\?[a-zA-Z-]*U|\\[0-9]")
_GO_S = r"\t\n\f\r "


def go_to_python(p: str):
    """A CPython pattern with Go's meaning for ASCII text, or None."""
    if _UNSUPPORTED.search(p):
        return None
    out = []
    # per open group: the scoped-flag string currently in force at this level ("" none)
    stack = [""]
    i, n = 0, len(p)
    in_cls = False
    while i < n:
        c = p[i]
        if c == "\\":
            if i + 1 >= n:
                return None
            e = p[i + 1]
            if in_cls:
                if e == "s":
                    out.append(_GO_S)
                elif e == "S":  # the complement of Go's \s as ranges (a class of a class)
                    out.append(r"\x00-\x08\x0b\x0e-\x1f\x21-\U0010ffff")
                else:
                    out.append(c + e)
            elif e == "s":
                out.append("[" + _GO_S + "]")
            elif e == "S":
                out.append("[^" + _GO_S + "]")
            elif e == "z":
                out.append(r"\Z")
            else:
                out.append(c + e)
            i += 2
            continue
        if in_cls:
            if c == "]":
                in_cls = False
            out.append(c)
            i += 1
            continue
        if c == "[":
            in_cls = True
            if p.startswith("[^", i):
                out.append("[^")
                i += 2
            else:
                out.append("[")
                i += 1
            if i < n and p[i] == "]":  # a leading ']' is a literal in both
                out.append("]")
                i += 1
            continue
        if c == "(":
            m = re.match(r"\(\?([a-z]*(?:-[a-z]*)?)\)", p[i:])
            if m:  # (?flags): the rest of this group, in every later alternative
                if stack[-1]:
                    out.append(")")
                fl = m.group(1)
                stack[-1] = fl
                out.append("(?%s:" % fl)
                i += m.end()
                continue
            stack.append("")
            out.append(c)
            i += 1
            continue
        if c == "|":
            if stack[-1]:
                out.append(")|(?%s:" % stack[-1])
            else:
                out.append("|")
            i += 1
            continue
        if c == ")":
            if len(stack) == 1:
                return None
            if stack.pop():
                out.append(")")
            out.append(")")
            i += 1
            continue
        out.append(c)
        i += 1
    if in_cls or len(stack) != 1:
        return None
    if stack[-1]:
        out.append(")")
    return "".join(out)


def _rx_args(text: str, files=None):
    cfg = coraza.parse_seclang(text, files)
    pats = []
    for r in cfg.rules:
        x = r
        while x is not None:
            if x.op is not None and x.op.name == "rx" and "%{" not in x.op.arg:
                pats.append(x.op.arg)
            x = x.chain
    return list(dict.fromkeys(pats))


def _patterns():
    pats = _rx_args(open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read())
    pats += [r[2] for r in gen_rxstress.rules()]
    c5_text, c5_files = traffic.c5_ruleset(n_rx=300, n_phrases=100)
    pats += _rx_args(c5_text, c5_files)
    return list(dict.fromkeys(pats))


def _corpus():
    vals, keep = set(), set()

    def add(v: bytes, crafted=False):
        if len(v) > 2048:
            return
        for w in (v, urllib.parse.unquote_to_bytes(v.replace(b"+", b" ")), v.lower()):
            if all(b < 0x80 for b in w):
                (keep if crafted else vals).add(w)
    g = traffic.TrafficGen(traffic.SEED + 77)
    parts, nh, _ = g.gen(300, post_frac=0.2, attack_rate=0.6)
    for p in parts:
        add(p)
        for a in re.split(rb"[?&;]", p):
            add(a)
            for kv in a.split(b"=", 1):
                add(kv)
    for p in traffic.ATTACKS:
        add(p, True)
        add(traffic._quote(p, True), True)
    for p in gen_rxstress.payloads(n=200):
        add(p, True)
    vocab, rules, phrases = traffic._c5_material(traffic.SEED, 300, 100)
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(5))
    for _ in range(300):
        add(b"x " + traffic._c5_snippet(rng, rules, phrases).lower() + b" y", True)
    add(b"a\x0bb\tc\nd\re f\x0c", True)
    # the crafted inputs whole, plus a seeded sample of the traffic-derived ones
    import random
    rest = sorted(vals - keep)
    return sorted(keep) + random.Random(3).sample(rest, min(len(rest), 5000))


@pytest.fixture(scope="module")
def material():
    return _patterns(), _corpus()


def test_translator_semantics():
    assert go_to_python(r"a(?i)b|c") == "a(?i:b)|(?i:c)"
    assert go_to_python(r"x\sy") == "x[" + _GO_S + "]y"
    assert go_to_python(r"\pL") is None and go_to_python(r"a{,3}") is None
    assert go_to_python(r"(a(?i)b)c") == "(a(?i:b))c"
    assert re.compile(go_to_python(r"[\s\S]x"), re.S).search("\x0bx")
    assert not re.compile(go_to_python(r"\sx"), re.S).search("\x0bx")  # Go's \s has no \v


def test_goregex_matches_cpython_on_stand_in_patterns(material):
    pats, corpus = material
    assert len(corpus) > 2000
    skipped, checked, positives, bad = [], 0, 0, []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for p in pats:
            t = go_to_python(p)
            if t is None:
                skipped.append(p)
                continue
            py = re.compile(t, re.S | re.M | re.A)
            go = goregex.rx_compile(p)
            checked += 1
            for v in corpus:
                a = go.match_string(v)
                b = py.search(v.decode("ascii")) is not None
                positives += a
                if a != b:
                    bad.append((p[:80], v[:80], a, b))
                    break
    assert not bad, bad[:10]
    # every stand-in pattern is translatable (nothing skipped silently)
    assert not skipped, skipped[:10]
    assert positives > 500  # the corpus reaches the patterns


def test_goregex_submatch_bounds_match_cpython(material):
    """FindStringSubmatch (capture: TX.0-TX.9) group boundaries on the
    capturing stand-in patterns: leftmost-first in both engines."""
    pats, corpus = material
    bad, n = [], 0
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for p in pats[:160]:
            t = go_to_python(p)
            if t is None:
                continue
            py = re.compile(t, re.S | re.M | re.A)
            go = goregex.rx_compile(p)
            for v in corpus[::3]:
                g = go.find_string_submatch(v)
                m = py.search(v.decode("ascii"))
                if (g is None) != (m is None):
                    bad.append((p[:60], v[:60]))
                    break
                if g is None:
                    continue
                n += 1
                want = [b"" if m.group(k) is None else m.group(k).encode("ascii") for k in range(len(g))]
                if g != want:
                    bad.append((p[:60], v[:60], g, want))
                    break
    assert not bad, bad[:5]
    assert n > 200
