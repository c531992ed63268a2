"""Go `regexp` (RE2) semantics restated in Python -- TEST INFRASTRUCTURE ONLY.

This module is part of the CPU oracle (`oracle/`).  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it,
and only as the checker: the product path (the HIP engine behind
`include/gpuinspect.h`) never calls into it.

What it restates
----------------
Coraza's `@rx` operator (coraza/v3 v3.3.3 `internal/operators/rx.go`
[upstream, not vendored in /root/reference; pinned by go.mod:6]) compiles
`"(?sm)" + pattern` with Go's `regexp` package and calls
`MatchString` / `FindStringSubmatch`.  Go's regexp parses patterns with
`regexp/syntax` Perl flags (ClassNL | OneLine | PerlX | UnicodeGroups) and
matches over *runes*: every byte sequence that is not valid UTF-8 decodes
as U+FFFD, one byte at a time (`utf8.DecodeRuneInString`).

The oracle parses the RE2 syntax itself (an independent parser from the
product's C++ one), expands every Go-specific construct into explicit,
flag-free Python `re` syntax -- `\\d \\s \\w` and `\\b` are ASCII-only,
`(?i)` is Unicode *simple* case folding (k ~ K ~ U+212A, s ~ S ~ U+017F),
`$` without (?m) is end-of-text only -- and then lets CPython's backtracking
engine do the matching.  For regular (back-reference-free) patterns a
backtracking leftmost-first engine and RE2 agree on both the boolean match
and the submatch boundaries, so Python's engine is an independent check of
the product's DFA construction.

Parity status: the parser follows Go's `regexp/syntax/parse.go` behaviour
as published for Go 1.22+; it is not pinned against a Go toolchain here
(none is installed).  `\\p{..}` Unicode groups are rejected (the product
rejects them too) and are "parity unpinned".
"""

from __future__ import annotations

import functools
import re
import unicodedata

MAX_RUNE = 0x10FFFF
MAX_REPEAT = 1000

# ---------------------------------------------------------------------------
# Go UTF-8 decoding (utf8.DecodeRune): invalid byte -> U+FFFD, width 1.
# ---------------------------------------------------------------------------


def go_decode(data: bytes) -> str:
    """Decode bytes into the rune sequence Go's regexp sees."""
    try:
        return data.decode("utf-8")  # strict == Go's notion of valid UTF-8
    except UnicodeDecodeError:
        pass
    out = []
    i, n = 0, len(data)
    while i < n:
        c = data[i]
        if c < 0x80:
            out.append(chr(c))
            i += 1
            continue
        r, w = _decode_rune(data, i)
        out.append(chr(r))
        i += w
    return "".join(out)


def _decode_rune(b: bytes, i: int):
    """Return (rune, width) following Go's utf8.DecodeRune acceptance table."""
    n = len(b)
    c0 = b[i]
    if c0 < 0x80:
        return c0, 1
    if 0xC2 <= c0 <= 0xDF:
        need, lo, hi = 1, 0x80, 0xBF
    elif c0 == 0xE0:
        need, lo, hi = 2, 0xA0, 0xBF
    elif 0xE1 <= c0 <= 0xEC or 0xEE <= c0 <= 0xEF:
        need, lo, hi = 2, 0x80, 0xBF
    elif c0 == 0xED:
        need, lo, hi = 2, 0x80, 0x9F
    elif c0 == 0xF0:
        need, lo, hi = 3, 0x90, 0xBF
    elif 0xF1 <= c0 <= 0xF3:
        need, lo, hi = 3, 0x80, 0xBF
    elif c0 == 0xF4:
        need, lo, hi = 3, 0x80, 0x8F
    else:
        return 0xFFFD, 1
    if n - i < need + 1:  # truncated sequence
        return 0xFFFD, 1
    if not (lo <= b[i + 1] <= hi):
        return 0xFFFD, 1
    for k in range(2, need + 1):
        if not (0x80 <= b[i + k] <= 0xBF):
            return 0xFFFD, 1
    seq = b[i:i + need + 1]
    return ord(seq.decode("utf-8")), need + 1


# ---------------------------------------------------------------------------
# Unicode simple case folding orbits (unicode.SimpleFold).
# ---------------------------------------------------------------------------


@functools.lru_cache(maxsize=None)
def _fold_tables():
    """orbit[c] -> sorted tuple of runes equivalent to c under simple folding."""
    key_members = {}
    for c in range(MAX_RUNE + 1):
        if 0xD800 <= c <= 0xDFFF:
            continue
        ch = chr(c)
        f = ch.casefold()
        if len(f) != 1:
            lo = ch.lower()
            f = lo if len(lo) == 1 else ch
        if f == ch and ch.upper() == ch and ch.lower() == ch:
            continue
        key_members.setdefault(f, set()).add(c)
    orbit = {}
    for f, members in key_members.items():
        members = set(members)
        members.add(ord(f))
        if len(members) < 2:
            continue
        t = tuple(sorted(members))
        for m in t:
            orbit[m] = t
    foldable = sorted(orbit)
    return orbit, foldable


def fold_orbit(c: int):
    orbit, _ = _fold_tables()
    return orbit.get(c, (c,))


# ---------------------------------------------------------------------------
# Rune-range sets
# ---------------------------------------------------------------------------


def _clean(ranges):
    rs = sorted(ranges)
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + 1:
            if hi > out[-1][1]:
                out[-1] = (out[-1][0], hi)
        else:
            out.append((lo, hi))
    return out


def _negate(ranges):
    rs = _clean(ranges)
    out = []
    nxt = 0
    for lo, hi in rs:
        if lo > nxt:
            out.append((nxt, lo - 1))
        nxt = hi + 1
    if nxt <= MAX_RUNE:
        out.append((nxt, MAX_RUNE))
    return out


def _fold_ranges(ranges):
    import bisect
    orbit, foldable = _fold_tables()
    out = list(ranges)
    for lo, hi in ranges:
        i = bisect.bisect_left(foldable, lo)
        while i < len(foldable) and foldable[i] <= hi:
            for m in orbit[foldable[i]]:
                out.append((m, m))
            i += 1
    return _clean(out)


PERL_GROUPS = {
    "d": [(0x30, 0x39)],
    "s": [(0x09, 0x0A), (0x0C, 0x0D), (0x20, 0x20)],
    "w": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
}

POSIX_GROUPS = {
    "alnum": [(0x30, 0x39), (0x41, 0x5A), (0x61, 0x7A)],
    "alpha": [(0x41, 0x5A), (0x61, 0x7A)],
    "ascii": [(0x00, 0x7F)],
    "blank": [(0x09, 0x09), (0x20, 0x20)],
    "cntrl": [(0x00, 0x1F), (0x7F, 0x7F)],
    "digit": [(0x30, 0x39)],
    "graph": [(0x21, 0x7E)],
    "lower": [(0x61, 0x7A)],
    "print": [(0x20, 0x7E)],
    "punct": [(0x21, 0x2F), (0x3A, 0x40), (0x5B, 0x60), (0x7B, 0x7E)],
    "space": [(0x09, 0x0D), (0x20, 0x20)],
    "upper": [(0x41, 0x5A)],
    "word": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
    "xdigit": [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66)],
}


class RegexError(ValueError):
    """Mirrors a `regexp/syntax` compile error (the rule fails to compile)."""


# ---------------------------------------------------------------------------
# Parser  (Go regexp/syntax, flags = Perl)
# AST nodes:
#   ('cls', ranges)                 one rune from the set
#   ('cat', [n...]) ('alt', [n...])
#   ('rep', n, min, max, greedy)    max == -1 -> unbounded
#   ('cap', index, n)
#   ('empty',)
#   ('assert', kind)  kind in bot eot bol eol wb nwb
# ---------------------------------------------------------------------------

FLAG_I, FLAG_M, FLAG_S, FLAG_U = 1, 2, 4, 8


class _Parser:
    def __init__(self, pattern: str):
        self.s = pattern
        self.i = 0
        self.ncap = 0

    def peek(self, k=0):
        j = self.i + k
        return self.s[j] if j < len(self.s) else None

    def eof(self):
        return self.i >= len(self.s)

    # alternation ---------------------------------------------------------
    def parse(self):
        flags = 0
        node = self.parse_alt(flags, top=True)
        if not self.eof():
            raise RegexError("unexpected )")
        return node

    def parse_alt(self, flags, top=False):
        branches = []
        box = [flags]
        while True:
            branches.append(self.parse_concat(box))
            if self.peek() == "|":
                self.i += 1
                continue
            break
        if len(branches) == 1:
            return branches[0]
        return ("alt", branches)

    def parse_concat(self, box):
        items = []
        while not self.eof():
            c = self.peek()
            if c == "|" or c == ")":
                break
            if c in "*+?":
                if not items or items[-1] is None:
                    raise RegexError("missing argument to repetition operator")
                self.i += 1
                lo, hi = {"*": (0, -1), "+": (1, -1), "?": (0, 1)}[c]
                self._apply_repeat(items, lo, hi, box[0])
                continue
            if c == "{":
                rep = self._try_brace()
                if rep is not None:
                    if not items or items[-1] is None:
                        raise RegexError("missing argument to repetition operator")
                    lo, hi = rep
                    self._apply_repeat(items, lo, hi, box[0])
                    continue
                # literal '{'
                self.i += 1
                items.append(self._lit(ord("{"), box[0]))
                self._last_rep = False
                continue
            self._last_rep = False
            atom = self.parse_atom(box)
            self._last_rep = False
            if atom is not None:
                items.append(atom)
        items = [x for x in items if x is not None]
        if not items:
            return ("empty",)
        if len(items) == 1:
            return items[0]
        return ("cat", items)

    _last_rep = False

    def _apply_repeat(self, items, lo, hi, flags):
        greedy = True
        if self.peek() == "?":
            self.i += 1
            greedy = False
        if self._last_rep:
            raise RegexError("invalid nested repetition operator")
        if flags & FLAG_U:
            greedy = not greedy
        if lo > MAX_REPEAT or hi > MAX_REPEAT or (hi != -1 and hi < lo):
            raise RegexError("invalid repeat count")
        items[-1] = ("rep", items[-1], lo, hi, greedy)
        self._last_rep = True

    def _try_brace(self):
        m = re.match(r"\{(\d+)(,(\d*))?\}", self.s[self.i:])
        if not m:
            return None
        for g in (m.group(1), m.group(3)):
            if g and len(g) > 1 and g[0] == "0":
                return None  # Go parseInt: no leading zeros
        lo = int(m.group(1))
        if m.group(2) is None:
            hi = lo
        elif m.group(3) == "":
            hi = -1
        else:
            hi = int(m.group(3))
        if len(m.group(1)) > 8 or (m.group(3) and len(m.group(3)) > 8):
            raise RegexError("invalid repeat count")
        if lo > MAX_REPEAT or hi > MAX_REPEAT or (hi != -1 and hi < lo):
            raise RegexError("invalid repeat count")
        self.i += m.end()
        return lo, hi

    # atoms -----------------------------------------------------------------
    def _lit(self, r, flags):
        if flags & FLAG_I:
            return ("cls", _fold_ranges([(r, r)]))
        return ("cls", [(r, r)])

    def parse_atom(self, box):
        flags = box[0]
        c = self.peek()
        if c == "(":
            return self.parse_group(box)
        if c == "[":
            return self.parse_class(flags)
        if c == ".":
            self.i += 1
            if flags & FLAG_S:
                return ("cls", [(0, MAX_RUNE)])
            return ("cls", [(0, 9), (11, MAX_RUNE)])
        if c == "^":
            self.i += 1
            return ("assert", "bol" if flags & FLAG_M else "bot")
        if c == "$":
            self.i += 1
            return ("assert", "eol" if flags & FLAG_M else "eot")
        if c == "\\":
            return self.parse_backslash(flags)
        self.i += 1
        return self._lit(ord(c), flags)

    def parse_group(self, box):
        s = self.s
        self.i += 1  # (
        flags = box[0]
        if self.peek() == "?":
            # named capture
            if s.startswith("?P<", self.i) or (s.startswith("?<", self.i) and not s.startswith("?<=", self.i) and not s.startswith("?<!", self.i)):
                start = self.i + (3 if s.startswith("?P<", self.i) else 2)
                end = s.find(">", start)
                if end < 0:
                    raise RegexError("invalid named capture")
                name = s[start:end]
                if not name or not re.fullmatch(r"[A-Za-z0-9_]+", name):
                    raise RegexError("invalid named capture")
                self.i = end + 1
                self.ncap += 1
                idx = self.ncap
                inner = self.parse_alt(flags)
                if self.peek() != ")":
                    raise RegexError("missing closing )")
                self.i += 1
                return ("cap", idx, inner)
            # flags
            j = self.i + 1
            sign = 1
            saw = False
            nf = flags
            while True:
                if j >= len(s):
                    raise RegexError("missing closing )")
                ch = s[j]
                if ch in "imsU":
                    bit = {"i": FLAG_I, "m": FLAG_M, "s": FLAG_S, "U": FLAG_U}[ch]
                    nf = (nf | bit) if sign > 0 else (nf & ~bit)
                    saw = True
                    j += 1
                    continue
                if ch == "-":
                    if sign < 0:
                        raise RegexError("invalid or unsupported Perl syntax")
                    sign = -1
                    saw = False
                    j += 1
                    continue
                if ch == ":" or ch == ")":
                    if sign < 0 and not saw:
                        raise RegexError("invalid or unsupported Perl syntax")
                    if ch == ")" and j == self.i + 1:
                        raise RegexError("invalid or unsupported Perl syntax")
                    break
                raise RegexError("invalid or unsupported Perl syntax")
            if s[j] == ")":
                # (?flags) -- applies to rest of current group
                self.i = j + 1
                box[0] = nf
                return None
            self.i = j + 1
            inner = self.parse_alt(nf)
            if self.peek() != ")":
                raise RegexError("missing closing )")
            self.i += 1
            return ("grp", inner)
        self.ncap += 1
        idx = self.ncap
        inner = self.parse_alt(flags)
        if self.peek() != ")":
            raise RegexError("missing closing )")
        self.i += 1
        return ("cap", idx, inner)

    def _perl_or_posix(self, name, neg, flags):
        rs = PERL_GROUPS[name] if len(name) == 1 else POSIX_GROUPS[name]
        if flags & FLAG_I:
            rs = _fold_ranges(rs)
        return _negate(rs) if neg else list(rs)

    def parse_backslash(self, flags):
        s = self.s
        if self.i + 1 >= len(s):
            raise RegexError("trailing backslash at end of expression")
        c = s[self.i + 1]
        if c == "A":
            self.i += 2
            return ("assert", "bot")
        if c == "z":
            self.i += 2
            return ("assert", "eot")
        if c == "b":
            self.i += 2
            return ("assert", "wb")
        if c == "B":
            self.i += 2
            return ("assert", "nwb")
        if c == "Q":
            end = s.find("\\E", self.i + 2)
            lit = s[self.i + 2:] if end < 0 else s[self.i + 2:end]
            self.i = len(s) if end < 0 else end + 2
            nodes = [self._lit(ord(ch), flags) for ch in lit]
            if not nodes:
                return None
            return nodes[0] if len(nodes) == 1 else ("cat", nodes)
        if c in "dswDSW":
            self.i += 2
            return ("cls", self._perl_or_posix(c.lower(), c.isupper(), flags))
        if c in "pP":
            raise RegexError("unsupported Unicode class escape")
        r = self.parse_escape()
        return self._lit(r, flags)

    def parse_escape(self):
        s = self.s
        assert s[self.i] == "\\"
        self.i += 1
        if self.i >= len(s):
            raise RegexError("trailing backslash at end of expression")
        c = s[self.i]
        self.i += 1
        oc = ord(c)
        if oc < 0x80 and not c.isalnum():
            return oc
        if c in "1234567":
            if self.i >= len(s) or not ("0" <= s[self.i] <= "7"):
                raise RegexError("invalid escape sequence")
        if c in "01234567":
            r = oc - 0x30
            for _ in range(2):
                if self.i < len(s) and "0" <= s[self.i] <= "7":
                    r = r * 8 + ord(s[self.i]) - 0x30
                    self.i += 1
                else:
                    break
            return r
        if c == "x":
            if self.i >= len(s):
                raise RegexError("invalid escape sequence")
            if s[self.i] == "{":
                end = s.find("}", self.i)
                if end < 0:
                    raise RegexError("invalid escape sequence")
                hx = s[self.i + 1:end]
                if not hx or not re.fullmatch(r"[0-9A-Fa-f]+", hx) or int(hx, 16) > MAX_RUNE:
                    raise RegexError("invalid escape sequence")
                self.i = end + 1
                return int(hx, 16)
            hx = s[self.i:self.i + 2]
            if len(hx) < 2 or not re.fullmatch(r"[0-9A-Fa-f]{2}", hx):
                raise RegexError("invalid escape sequence")
            self.i += 2
            return int(hx, 16)
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if c in simple:
            return simple[c]
        raise RegexError("invalid escape sequence")

    def parse_class(self, flags):
        s = self.s
        self.i += 1  # [
        neg = False
        if self.peek() == "^":
            neg = True
            self.i += 1
        ranges = []
        first = True
        while True:
            if self.eof():
                raise RegexError("missing closing ]")
            c = self.peek()
            if c == "]" and not first:
                self.i += 1
                break
            first = False
            if s.startswith("[:", self.i):
                end = s.find(":]", self.i + 2)
                if end >= 0:
                    name = s[self.i + 2:end]
                    pneg = name.startswith("^")
                    if pneg:
                        name = name[1:]
                    if name not in POSIX_GROUPS:
                        raise RegexError("invalid character class range")
                    ranges += self._perl_or_posix(name, pneg, flags)
                    self.i = end + 2
                    continue
            if c == "\\" and self.peek(1) in ("d", "s", "w", "D", "S", "W"):
                k = self.peek(1)
                ranges += self._perl_or_posix(k.lower(), k.isupper(), flags)
                self.i += 2
                continue
            if c == "\\" and self.peek(1) in ("p", "P"):
                raise RegexError("unsupported Unicode class escape")
            lo = self._class_char()
            hi = lo
            if self.peek() == "-" and self.peek(1) is not None and self.peek(1) != "]":
                self.i += 1
                hi = self._class_char()
                if hi < lo:
                    raise RegexError("invalid character class range")
            if flags & FLAG_I:
                ranges += _fold_ranges([(lo, hi)])
            else:
                ranges.append((lo, hi))
        ranges = _clean(ranges)
        if neg:
            ranges = _negate(ranges)
        return ("cls", ranges)

    def _class_char(self):
        c = self.peek()
        if c == "\\":
            return self.parse_escape()
        self.i += 1
        return ord(c)


def parse(pattern: str):
    """Parse an RE2 pattern (Go regexp/syntax, Perl flags) into an AST."""
    p = _Parser(pattern)
    node = p.parse()
    return node, p.ncap


# ---------------------------------------------------------------------------
# Translation to flag-free Python `re`
# ---------------------------------------------------------------------------

_W = "0-9A-Za-z_"
_ASSERT_PY = {
    "bot": r"\A",
    "eot": r"\Z",
    "bol": r"(?:\A|(?<=\n))",
    "eol": r"(?=\n|\Z)",
    "wb": r"(?:(?<=[%s])(?![%s])|(?<![%s])(?=[%s]))" % (_W, _W, _W, _W),
    "nwb": r"(?:(?<=[%s])(?=[%s])|(?<![%s])(?![%s]))" % (_W, _W, _W, _W),
}


def _esc(c: int) -> str:
    return "\\U%08x" % c


def _emit(node) -> str:
    kind = node[0]
    if kind == "cls":
        rs = node[1]
        if not rs:
            return "(?!)"
        parts = []
        for lo, hi in rs:
            parts.append(_esc(lo) if lo == hi else _esc(lo) + "-" + _esc(hi))
        return "[" + "".join(parts) + "]"
    if kind == "cat":
        return "".join(_emit(n) for n in node[1])
    if kind == "alt":
        return "(?:" + "|".join(_emit(n) for n in node[1]) + ")"
    if kind == "grp":
        return "(?:" + _emit(node[1]) + ")"
    if kind == "cap":
        return "(" + _emit(node[2]) + ")"
    if kind == "rep":
        _, sub, lo, hi, greedy = node
        inner = "(?:" + _emit(sub) + ")"
        if lo == 0 and hi == -1:
            q = "*"
        elif lo == 1 and hi == -1:
            q = "+"
        elif lo == 0 and hi == 1:
            q = "?"
        elif hi == -1:
            q = "{%d,}" % lo
        elif lo == hi:
            q = "{%d}" % lo
        else:
            q = "{%d,%d}" % (lo, hi)
        return inner + q + ("" if greedy else "?")
    if kind == "empty":
        return "(?:)"
    if kind == "assert":
        return _ASSERT_PY[node[1]]
    raise AssertionError(kind)


def _required(node):
    """A necessary condition of a match as literal strings: every match
    contains at least one of them (None: no condition).  Only exact single-rune
    classes form literals, so the condition never rejects a matching text; it
    lets the oracle skip the backtracking search on most texts of large
    generated rulesets (C5).  Speed only: the result is unchanged."""
    kind = node[0]
    if kind == "cls":
        rs = node[1]
        if len(rs) == 1 and rs[0][0] == rs[0][1]:
            return {chr(rs[0][0])}
        return None
    if kind in ("grp",):
        return _required(node[1])
    if kind == "cap":
        return _required(node[2])
    if kind == "rep":
        return _required(node[1]) if node[2] >= 1 else None
    if kind == "alt":
        out = set()
        for k in node[1]:
            r = _required(k)
            if r is None:
                return None
            out |= r
        return out
    if kind == "cat":
        best = None

        def better(c):
            return best is None or min(map(len, c)) > min(map(len, best)) or (
                min(map(len, c)) == min(map(len, best)) and len(c) < len(best))
        run = ""
        for k in node[1]:
            if k[0] == "cls" and len(k[1]) == 1 and k[1][0][0] == k[1][0][1]:
                run += chr(k[1][0][0])
                continue
            if run and better({run}):
                best = {run}
            run = ""
            r = _required(k)
            if r is not None and better(r):
                best = r
        if run and better({run}):
            best = {run}
        return best
    return None


class GoRegexp:
    """A compiled Go regexp evaluated with CPython's engine on Go runes."""

    def __init__(self, pattern: str):
        self.pattern = pattern
        ast, ncap = parse(pattern)
        self.ncap = ncap
        self.py = re.compile(_emit(ast))
        req = _required(ast)
        self.req = tuple(req) if req and all(req) else None

    def _may_match(self, text: str) -> bool:
        return self.req is None or any(r in text for r in self.req)

    def match_string(self, data: bytes) -> bool:
        text = go_decode(data)
        return self._may_match(text) and self.py.search(text) is not None

    def find_string_submatch(self, data: bytes):
        """Go's FindStringSubmatch: list of group strings (bytes) or None."""
        text = go_decode(data)
        if not self._may_match(text):
            return None
        m = self.py.search(text)
        if m is None:
            return None
        # Group offsets are in runes; map back to the original bytes.
        offs = _rune_offsets(data, text)
        out = []
        for g in range(self.ncap + 1):
            sp = m.span(g)
            if sp[0] < 0:
                out.append(b"")
            else:
                out.append(data[offs[sp[0]]:offs[sp[1]]])
        return out


def _rune_offsets(data: bytes, text: str):
    """Byte offset of every rune boundary (len(text)+1 entries)."""
    offs = [0] * (len(text) + 1)
    i = 0
    n = len(data)
    for k in range(len(text)):
        offs[k] = i
        c = data[i]
        if c < 0x80:
            i += 1
        else:
            _, w = _decode_rune(data, i)
            i += w
    offs[len(text)] = n
    return offs


@functools.lru_cache(maxsize=8192)
def compile_go(pattern: str) -> GoRegexp:
    return GoRegexp(pattern)


def rx_compile(arg: str) -> GoRegexp:
    """Coraza @rx: `regexp.Compile("(?sm)" + arg)` [upstream rx.go]."""
    return compile_go("(?sm)" + arg)
