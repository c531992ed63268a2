"""Coraza's XML body processor restated -- TEST INFRASTRUCTURE ONLY.

Part of the CPU oracle (`oracle/`): only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline / parity leg use it, as the checker.

[upstream coraza/v3 v3.3.3 internal/bodyprocessors/xml.go, not vendored in
/root/reference; pinned by go.mod:6] readXML runs Go's encoding/xml Decoder
with Strict = false, AutoClose = xml.HTMLAutoClose, Entity = xml.HTMLEntity
and keeps, in document order,
  * every attribute value of every StartElement      -> XML "//@*"
  * every CharData token, strings.TrimSpace'd, if not empty -> XML "/*"
A Token() error other than io.EOF fails the processor: no XML values,
REQBODY_ERROR "1", REQBODY_ERROR_MSG "XML: " + err.Error().

This module restates the Decoder paths that produces (Go encoding/xml
xml.go: rawToken, text, attrval, name / nsname, autoClose, popElement, the
<?xml?> version / encoding checks, SyntaxError's "XML syntax error on line
N: msg").  Names with non-ASCII bytes need Go's XML NameStartChar / NameChar
range tables: such bodies raise XmlUnsupported (an engine limit the GPU flags
the same way).  Parity status: restated from the published Go sources;
unpinned (no Go toolchain here).
"""

from __future__ import annotations

import html.entities

AUTO_CLOSE = ("basefont", "br", "area", "link", "img", "param", "hr", "input", "col", "frame", "isindex", "base",
              "meta")  # xml.HTMLAutoClose
XML_ENTITY = {"lt": "<", "gt": ">", "amp": "&", "apos": "'", "quot": '"'}
# xml.HTMLEntity: the HTML 4.01 character entities
HTML_ENTITY = {k: chr(v) for k, v in html.entities.name2codepoint.items()}

# unicode.IsSpace (strings.TrimSpace)
_SPACE = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2000, 0x2001, 0x2002, 0x2003, 0x2004, 0x2005,
          0x2006, 0x2007, 0x2008, 0x2009, 0x200A, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000}


class XmlError(Exception):
    """Decoder.Token() error (the processor's error text)."""


class XmlUnsupported(Exception):
    """Input outside the engine's restatement (non-ASCII XML names)."""


def _name_byte(c: int) -> bool:
    return (65 <= c <= 90) or (97 <= c <= 122) or (48 <= c <= 57) or c in (0x5F, 0x3A, 0x2E, 0x2D)


def _in_char_range(r: int) -> bool:
    return r in (0x09, 0x0A, 0x0D) or 0x20 <= r <= 0xD7FF or 0xE000 <= r <= 0xFFFD or 0x10000 <= r <= 0x10FFFF


def _decode_rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, size); invalid -> (0xFFFD, 1)."""
    from .goregex import _decode_rune as dr
    return dr(b, i)


def trim_space(b: bytes) -> bytes:
    """strings.TrimSpace over UTF-8 (invalid bytes are not space)."""
    i, n = 0, len(b)
    while i < n:
        r, w = _decode_rune(b, i)
        if (r == 0xFFFD and w == 1) or r not in _SPACE:
            break
        i += w
    j = n
    while j > i:
        # step back one rune (Go: utf8.DecodeLastRune)
        k = j - 1
        while k > i and j - k < 4 and (b[k] & 0xC0) == 0x80:
            k -= 1
        r, w = _decode_rune(b, k)
        if k + w != j:  # not a whole rune ending at j: the last byte alone is invalid
            k, r, w = j - 1, 0xFFFD, 1
        if (r == 0xFFFD and w == 1) or r not in _SPACE:
            break
        j = k
    return b[i:j]


class _Dec:
    def __init__(self, data: bytes):
        self.s = data
        self.i = 0
        self.line = 1
        self.stk = []          # open element names: (space, local)
        self.need_close = False
        self.to_close = None
        self.next_tok = None

    # -- bytes ---------------------------------------------------------------
    def getc(self):
        if self.i >= len(self.s):
            return None
        b = self.s[self.i]
        self.i += 1
        if b == 0x0A:
            self.line += 1
        return b

    def ungetc(self, b):
        if b == 0x0A:
            self.line -= 1
        self.i -= 1

    def syntax(self, msg):
        return XmlError("XML syntax error on line %d: %s" % (self.line, msg))

    def mustgetc(self):
        b = self.getc()
        if b is None:
            raise self.syntax("unexpected EOF")
        return b

    def space(self):
        while True:
            b = self.getc()
            if b is None:
                return
            if b not in (0x20, 0x0D, 0x0A, 0x09):
                self.ungetc(b)
                return

    # -- names ---------------------------------------------------------------
    def read_name(self, buf: bytearray) -> bool:
        b = self.mustgetc()
        if b < 0x80 and not _name_byte(b):
            self.ungetc(b)
            return False
        buf.append(b)
        while True:
            b = self.mustgetc()
            if b < 0x80 and not _name_byte(b):
                self.ungetc(b)
                break
            buf.append(b)
        return True

    def is_name(self, b: bytes) -> bool:
        if not b:
            return False
        if any(c >= 0x80 for c in b):
            raise XmlUnsupported("non-ASCII XML name")
        c = b[0]
        if not ((65 <= c <= 90) or (97 <= c <= 122) or c in (0x5F, 0x3A)):
            return False
        return True  # ASCII name bytes after the first are all NameChar

    def name(self):
        buf = bytearray()
        if not self.read_name(buf):
            return None
        if not self.is_name(bytes(buf)):
            raise self.syntax("invalid XML name: " + buf.decode("latin-1"))
        return bytes(buf)

    def nsname(self):
        s = self.name()
        if s is None:
            return None
        if s.count(b":") > 1:
            return None
        sp, sep, loc = s.partition(b":")
        if not sep or not sp or not loc:
            return (b"", s)
        return (sp, loc)

    # -- text ----------------------------------------------------------------
    def text(self, quote: int, cdata: bool) -> bytes:
        b0 = b1 = 0
        trunc = 0
        buf = bytearray()
        while True:
            b = self.getc()
            if b is None:
                if cdata:
                    raise self.syntax("unexpected EOF in CDATA section")
                break
            if quote < 0 and b0 == 0x5D and b1 == 0x5D and b == 0x3E:
                if cdata:
                    trunc = 2
                    break
                raise self.syntax("unescaped ]]> not in CDATA section")
            if b == 0x3C and not cdata:
                if quote >= 0:
                    raise self.syntax("unescaped < inside quoted string")
                self.ungetc(b)
                break
            if quote >= 0 and b == quote:
                break
            if b == 0x26 and not cdata:
                before = len(buf)
                buf.append(0x26)
                text = None
                b = self.mustgetc()
                if b == 0x23:  # '#'
                    buf.append(b)
                    b = self.mustgetc()
                    base = 10
                    if b == 0x78:  # 'x'
                        base = 16
                        buf.append(b)
                        b = self.mustgetc()
                    start = len(buf)
                    while (48 <= b <= 57) or (base == 16 and (97 <= b <= 102 or 65 <= b <= 70)):
                        buf.append(b)
                        b = self.mustgetc()
                    if b != 0x3B:
                        self.ungetc(b)
                    else:
                        digits = bytes(buf[start:])
                        buf.append(0x3B)
                        if digits:
                            n = int(digits, base)
                            if n <= 0x10FFFF:
                                text = chr(n) if not (0xD800 <= n <= 0xDFFF) else "�"
                else:
                    self.ungetc(b)
                    self.read_name(buf)  # (no error when it reads nothing)
                    b = self.mustgetc()
                    if b != 0x3B:
                        self.ungetc(b)
                    else:
                        nm = bytes(buf[before + 1:])
                        buf.append(0x3B)
                        # isName(nm): both entity maps have ASCII keys only, so a
                        # name with non-ASCII bytes never substitutes either way
                        if nm and all(c < 0x80 for c in nm) and self.is_name(nm):
                            s = nm.decode("ascii")
                            if s in XML_ENTITY:
                                text = XML_ENTITY[s]
                            elif s in HTML_ENTITY:
                                text = HTML_ENTITY[s]
                if text is not None:
                    del buf[before:]
                    buf += text.encode("utf-8", "surrogatepass")
                b0 = b1 = 0
                continue  # (non-strict: an unknown entity stays as written)
            if b == 0x0D:
                buf.append(0x0A)
            elif b1 == 0x0D and b == 0x0A:
                pass
            else:
                buf.append(b)
            b0, b1 = b1, b
        data = bytes(buf[:len(buf) - trunc])
        i = 0
        while i < len(data):
            r, w = _decode_rune(data, i)
            if r == 0xFFFD and w == 1:
                raise self.syntax("invalid UTF-8")
            i += w
            if not _in_char_range(r):
                raise self.syntax("illegal character code U+%04X" % r)
        return data

    def attrval(self) -> bytes:
        b = self.mustgetc()
        if b in (0x22, 0x27):
            return self.text(b, False)
        self.ungetc(b)
        buf = bytearray()
        while True:
            b = self.mustgetc()
            if (97 <= b <= 122) or (65 <= b <= 90) or (48 <= b <= 57) or b in (0x5F, 0x3A, 0x2D):
                buf.append(b)
            else:
                self.ungetc(b)
                break
        return bytes(buf)

    # -- tokens --------------------------------------------------------------
    def raw_token(self):
        """('start', name, [attr values]) | ('end', name) | ('chars', bytes) |
        ('other',) | None at EOF."""
        if self.need_close:
            self.need_close = False
            return ("end", self.to_close)
        b = self.getc()
        if b is None:
            return None
        if b != 0x3C:
            self.ungetc(b)
            return ("chars", self.text(-1, False))
        b = self.mustgetc()
        if b == 0x2F:  # </
            name = self.nsname()
            if name is None:
                raise self.syntax("expected element name after </")
            self.space()
            b = self.mustgetc()
            if b != 0x3E:
                raise self.syntax("invalid characters between </" + name[1].decode() + " and >")
            return ("end", name)
        if b == 0x3F:  # <?
            target = self.name()
            if target is None:
                raise self.syntax("expected target name after <?")
            self.space()
            buf = bytearray()
            b0 = 0
            while True:
                b = self.mustgetc()
                buf.append(b)
                if b0 == 0x3F and b == 0x3E:
                    break
                b0 = b
            content = bytes(buf[:-2])
            if target == b"xml":
                ver = _proc_inst(b"version", content)
                if ver and ver != b"1.0":
                    raise XmlError('xml: unsupported version "%s"; only version 1.0 is supported' % ver.decode("latin-1"))
                enc = _proc_inst(b"encoding", content)
                if enc and enc.lower() != b"utf-8":
                    raise XmlError('xml: encoding "%s" declared but Decoder.CharsetReader is nil' % enc.decode("latin-1"))
            return ("other",)
        if b == 0x21:  # <!
            b = self.mustgetc()
            if b == 0x2D:  # <!-
                b = self.mustgetc()
                if b != 0x2D:
                    raise self.syntax("invalid sequence <!- not part of <!--")
                b0 = b1 = 0
                while True:
                    b = self.mustgetc()
                    if b0 == 0x2D and b1 == 0x2D:
                        if b != 0x3E:
                            raise self.syntax('invalid sequence "--" not allowed in comments')
                        break
                    b0, b1 = b1, b
                return ("other",)
            if b == 0x5B:  # <![
                for c in b"CDATA[":
                    if self.mustgetc() != c:
                        raise self.syntax("invalid <![ sequence")
                return ("chars", self.text(-1, True))
            # a directive: quoted '>' and nested <...> / comments skipped
            inquote = 0
            depth = 0
            while True:
                b = self.mustgetc()
                if inquote == 0 and b == 0x3E and depth == 0:
                    break
                while True:  # HandleB
                    if b == inquote:
                        inquote = 0
                    elif inquote != 0:
                        pass
                    elif b in (0x27, 0x22):
                        inquote = b
                    elif b == 0x3E:
                        depth -= 1
                    elif b == 0x3C:
                        redo = False
                        for k, c in enumerate(b"!--"):
                            b = self.mustgetc()
                            if b != c:
                                depth += 1
                                redo = True
                                break
                        if redo:
                            continue  # goto HandleB with this byte
                        b0 = b1 = 0
                        while True:
                            b = self.mustgetc()
                            if b0 == 0x2D and b1 == 0x2D and b == 0x3E:
                                break
                            b0, b1 = b1, b
                    break
            return ("other",)
        # an open element
        self.ungetc(b)
        name = self.nsname()
        if name is None:
            raise self.syntax("expected element name after <")
        attrs = []
        empty = False
        while True:
            self.space()
            b = self.mustgetc()
            if b == 0x2F:
                empty = True
                b = self.mustgetc()
                if b != 0x3E:
                    raise self.syntax("expected /> in element")
                break
            if b == 0x3E:
                break
            self.ungetc(b)
            an = self.nsname()
            if an is None:
                raise self.syntax("expected attribute name in element")
            self.space()
            b = self.mustgetc()
            if b != 0x3D:
                self.ungetc(b)
                attrs.append(an[1])
            else:
                self.space()
                attrs.append(self.attrval())
        if empty:
            self.need_close = True
            self.to_close = name
        return ("start", name, attrs)

    def token(self):
        if self.next_tok is not None:
            t, self.next_tok = self.next_tok, None
        else:
            t = self.raw_token()
            if t is None:
                if self.stk:
                    raise self.syntax("unexpected EOF")
                return None
        # autoClose
        if self.stk and self.stk[-1][1].lower().decode("latin-1") in AUTO_CLOSE:
            top = self.stk[-1]
            if not (t[0] == "end" and t[1][1].lower() == top[1].lower()):
                self.next_tok = t
                t = ("end", top)
        if t[0] == "start":
            self.stk.append(t[1])
        elif t[0] == "end":
            name = t[1]
            if not self.stk:
                raise self.syntax("unexpected end element </" + name[1].decode("latin-1") + ">")
            s = self.stk.pop()
            if s[1] != name[1]:
                self.need_close = True
                self.to_close = name
            elif s[0] != name[0]:
                ns = name[0].decode("latin-1") or '""'
                raise self.syntax("element <%s> in space %s closed by </%s> in space %s" % (
                    s[1].decode("latin-1"), s[0].decode("latin-1"), name[1].decode("latin-1"), ns))
        return t


def _proc_inst(param: bytes, s: bytes) -> bytes:
    """encoding/xml procInst: the value of param="..." / param='...' or b""."""
    param = param + b"="
    lenp = len(param)
    i = 0
    sep = 0
    while i < len(s):
        sub = s[i:]
        k = sub.find(param)
        if k < 0 or lenp + k >= len(sub):
            return b""
        i += lenp + k + 1
        c = sub[lenp + k]
        if c in (0x27, 0x22):
            sep = c
            break
    if sep == 0:
        return b""
    j = s.find(bytes([sep]), i)
    if j < 0:
        return b""
    return s[i:j]


def read_xml(body: bytes):
    """readXML: (attribute values, trimmed non-empty character data).
    Raises XmlError (the processor's error) or XmlUnsupported."""
    d = _Dec(body)
    attrs, content = [], []
    while True:
        t = d.token()
        if t is None:
            break
        if t[0] == "start":
            attrs += t[2]
        elif t[0] == "chars":
            c = trim_space(t[1])
            if c:
                content.append(c)
    return attrs, content
