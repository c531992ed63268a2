"""The engine's Unicode case tables (csrc/unicode_tables.h, generated from
Perl's Unicode::UCD by tools/gen_unicode_tables.py) against the oracle's own
derivation (oracle/goregex.py: CPython str.casefold / str.lower).  The two
derivations share no code, so a wrong fold orbit or lowercase entry on either
side fails here.  Both are Unicode 13.0; Go 1.26 is Unicode 15.0 (runes
assigned or re-cased in 14.0/15.0: parity unpinned)."""
import os
import re

from oracle import goregex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "coraza-kubernetes-operator_amd", "csrc", "unicode_tables.h")


def _tables():
    s = open(HDR).read()
    b = s.index("GI_N_LOWER_PAIRS")
    pat = r"\{0x([0-9a-f]+),0x([0-9a-f]+)\}"
    fold = [(int(a, 16), int(c, 16)) for a, c in re.findall(pat, s[:b])]
    lower = [(int(a, 16), int(c, 16)) for a, c in re.findall(pat, s[b:])]
    return fold, lower


def test_fold_orbits_agree_with_oracle():
    fold, _ = _tables()
    orbit, foldable = goregex._fold_tables()
    eng = {}
    for a, b in fold:
        eng.setdefault(a, {a}).add(b)
    assert sorted(eng) == foldable
    for c, members in eng.items():
        assert tuple(sorted(members)) == orbit[c], hex(c)


def test_lowercase_agrees_with_cpython():
    _, lower = _tables()
    want = {}
    for c in range(0x110000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        lo = chr(c).lower()
        if len(lo) == 1 and ord(lo) != c:
            want[c] = ord(lo)
    want[0x130] = 0x69  # U+0130: full lowercase is 2 runes, the simple mapping is 'i'
    assert dict(lower) == want
    assert sorted(lower) == lower
