"""CPU restatement of coraza's MULTIPART body processor (test infrastructure:
only tests/, smoke() and bench.py's cpu_baseline leg use it).

[upstream coraza v3.3.3 internal/bodyprocessors/multipart.go, not vendored
under /root/reference]: ProcessRequest runs Go's mime.ParseMediaType on the
Content-Type, then mime/multipart.Reader.NextPart over the body:

  * a part whose Content-Disposition has a filename parameter is a file:
    FILES += ("", filename), FILES_SIZES.SetIndex(filename, 0, size),
    FILES_NAMES += ("", part name); the data is discarded (no upload
    storage: FILES_TMPNAMES stays empty, as under coraza's no-filesystem
    build used by proxy-wasm);
  * any other part is a field: ARGS_POST += (part name, data);
  * every header of a part: MULTIPART_PART_HEADERS += (part name,
    "Key: value") -- Go iterates the part's header map in random order; this
    restatement (and the device) use sorted canonical keys;
  * FILES_COMBINED_SIZE = running total of part sizes (set after each part);
  * a NextPart / read error: MULTIPART_STRICT_ERROR = "1" and the error is
    returned (the transaction sets REQBODY_ERROR); the collections keep what
    the parts before the error added.

Go semantics restated (parity unpinned: no Go toolchain or coraza source
here; anchored on the CRS base rules 200002/200003 in
/root/reference/hack/generate_coreruleset_configmaps.py:73-89):
  * mime.ParseMediaType: token media type, ';'-separated token=token or
    token="quoted" params, lowercased names, duplicate name = error; RFC 2231
    continuations/charsets are outside this engine (UnsupportedInput);
  * multipart.Reader: the delimiter is "--" + boundary; lines before the
    first delimiter are skipped (a line over 4096 bytes is bufio's "buffer
    full" error); a first delimiter line ending in a bare LF switches the
    reader to LF mode; a part's data ends at the first NL + "--" + boundary
    followed by space, tab, CR, LF, "--" or the end of the body; between
    parts only the NL itself may appear; "--boundary--" (+ LWSP, + NL) ends
    the body; running out of body before it is an error;
  * textproto.ReadMIMEHeader: header lines until a blank line, continuation
    lines (leading space / tab) joined with one space, keys canonicalised
    (invalid key bytes or a missing colon are an error), values trimmed;
  * Content-Transfer-Encoding: quoted-printable parts are decoded by Go
    before the processor sees them: outside this engine (UnsupportedInput).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple


class MultipartUnsupported(Exception):
    """Input this restatement (and the device) does not model."""


class MultipartError(Exception):
    """A Go error from ParseMediaType / NextPart / reading a part."""


TSPECIALS = set(b'()<>@,;:\\"/[]?=')


def _is_token_byte(c: int) -> bool:
    return 0x20 < c < 0x7F and c not in TSPECIALS


def _skip_ws(s: bytes, i: int) -> int:
    while i < len(s) and s[i] in b" \t":
        i += 1
    return i


def parse_media_type(v: bytes) -> Tuple[bytes, Dict[bytes, bytes]]:
    """Go mime.ParseMediaType (the subset above).  Raises MultipartError."""
    semi = v.find(b";")
    base = (v if semi < 0 else v[:semi]).strip(b" \t").lower()
    if not base:
        raise MultipartError("mime: no media type")
    # checkMediaTypeDisposition: token, optionally "/" token
    typ, slash, sub = base.partition(b"/")
    if not typ or not all(_is_token_byte(c) for c in typ):
        raise MultipartError("mime: expected token after slash" if slash else "mime: invalid media type")
    if slash and (not sub or not all(_is_token_byte(c) for c in sub)):
        raise MultipartError("mime: expected token after slash")
    params: Dict[bytes, bytes] = {}
    if semi < 0:
        return base, params
    rest = v[semi:]
    while True:
        rest = rest.lstrip(b" \t")
        if not rest:
            break
        if rest[0:1] != b";":
            raise MultipartError("mime: invalid media parameter")
        rest = rest[1:]
        i = _skip_ws(rest, 0)
        if i == len(rest):  # trailing ';'
            break
        j = i
        while j < len(rest) and _is_token_byte(rest[j]):
            j += 1
        key = rest[i:j].lower()
        if not key:
            raise MultipartError("mime: invalid media parameter")
        if b"*" in key:
            raise MultipartUnsupported("RFC 2231 parameter")
        j = _skip_ws(rest, j)
        if j >= len(rest) or rest[j] != ord("="):
            raise MultipartError("mime: invalid media parameter")
        j = _skip_ws(rest, j + 1)
        if j < len(rest) and rest[j] == ord('"'):
            k = j + 1
            val = bytearray()
            while k < len(rest) and rest[k] != ord('"'):
                if rest[k] in b"\r\n":
                    raise MultipartError("mime: invalid media parameter")
                if rest[k] == ord("\\") and k + 1 < len(rest) and rest[k + 1] in TSPECIALS:
                    k += 1  # consumeValue: a backslash escapes a tspecial only
                val.append(rest[k])
                k += 1
            if k >= len(rest):
                raise MultipartError("mime: invalid media parameter")
            value = bytes(val)
            k += 1
        else:
            k = j
            while k < len(rest) and _is_token_byte(rest[k]):
                k += 1
            value = rest[j:k]
            if not value:
                raise MultipartError("mime: invalid media parameter")
        if key in params:
            raise MultipartError("mime: duplicate parameter name")
        params[key] = value
        rest = rest[k:]
    return base, params


def _canonical_key(k: bytes) -> Optional[bytes]:
    """textproto.CanonicalMIMEHeaderKey with the validity check (None: invalid)."""
    if not k or not all(_is_token_byte(c) for c in k):
        return None
    out = bytearray()
    upper = True
    for c in k:
        if upper and 0x61 <= c <= 0x7A:
            c -= 32
        elif not upper and 0x41 <= c <= 0x5A:
            c += 32
        out.append(c)
        upper = c == ord("-")
    return bytes(out)


def _read_line(body: bytes, i: int) -> Tuple[Optional[bytes], int]:
    """A line without its NL (None at the end of the body)."""
    if i >= len(body):
        return None, i
    j = body.find(b"\n", i)
    if j < 0:
        return body[i:], len(body)
    line = body[i:j]
    if line.endswith(b"\r"):
        line = line[:-1]
    return line, j + 1


def read_mime_header(body: bytes, i: int) -> Tuple[List[Tuple[bytes, bytes]], int]:
    """textproto.ReadMIMEHeader from body[i:]: ([(canonical key, value)], next index)."""
    out: List[Tuple[bytes, bytes]] = []
    first = True
    while True:
        line, i = _read_line(body, i)
        if line is None:
            raise MultipartError("unexpected EOF")
        if first and line[:1] in (b" ", b"\t"):
            raise MultipartError("malformed MIME header initial line")
        first = False
        if line == b"":
            return out, i
        kv = line.strip(b" \t")
        # continuation lines
        while i < len(body) and body[i:i + 1] in (b" ", b"\t"):
            cont, i = _read_line(body, i)
            kv = kv + b" " + cont.strip(b" \t")
        k, colon, v = kv.partition(b":")
        if not colon:
            raise MultipartError("malformed MIME header line")
        key = _canonical_key(k)
        if key is None:
            raise MultipartError("malformed MIME header line")
        for c in v:
            if not (c >= 0x20 or c == 0x09) or c == 0x7F:
                raise MultipartError("malformed MIME header line")
        out.append((key, v.lstrip(b" \t")))


def _header_get(h, key: bytes) -> bytes:
    for k, v in h:
        if k == key:
            return v
    return b""


def _disposition(h) -> Tuple[bytes, Dict[bytes, bytes]]:
    try:
        return parse_media_type(_header_get(h, b"Content-Disposition"))
    except MultipartError:
        return b"", {}


def process(body: bytes, content_type: bytes):
    """coraza's multipart ProcessRequest over a whole body.

    Returns dict(args_post, files, files_names, files_sizes, part_headers,
    combined_size (bytes or None), error (str or None))."""
    res = {"args_post": [], "files": [], "files_names": [], "files_sizes": [], "part_headers": [],
           "combined_size": None, "error": None}
    try:
        mt, params = parse_media_type(content_type)
    except MultipartError:
        res["error"] = "mime: invalid media type"
        return res
    if not mt.startswith(b"multipart/"):
        res["error"] = "not a multipart body"
        return res
    boundary = params.get(b"boundary", b"")
    if boundary == b"":
        res["error"] = "multipart: boundary is empty"
        return res
    dash = b"--" + boundary
    nl = b"\r\n"
    parts_read = 0
    total = 0
    i = 0
    n = len(body)
    while True:
        # Reader.nextPart: lines until a delimiter line
        expect_new = False
        while True:
            j = body.find(b"\n", i)
            if j < 0 or j - i + 1 > 4096:
                if j < 0 and n - i < 4096:  # bufio: 4096 bytes without a NL fill the buffer
                    line = body[i:]
                    if _is_final(line, dash, nl):
                        return res
                    res["error"] = "multipart: NextPart: EOF"
                else:
                    res["error"] = "multipart: NextPart: bufio: buffer full"
                return res
            line = body[i:j + 1]
            i = j + 1
            if line.startswith(dash):
                rest = line[len(dash):].lstrip(b" \t")
                if parts_read == 0 and rest == b"\n":
                    nl = b"\n"
                if rest == nl:
                    break
            if _is_final(line, dash, nl):
                return res
            if expect_new:
                res["error"] = "multipart: expecting a new Part"
                return res
            if parts_read == 0:
                continue
            if line == nl:
                expect_new = True
                continue
            res["error"] = "multipart: unexpected line in Next()"
            return res
        parts_read += 1
        try:
            hdr, i = read_mime_header(body, i)
        except MultipartError:
            res["error"] = "multipart: NextPart: malformed MIME header"
            return res
        if _header_get(hdr, b"Content-Transfer-Encoding").lower() == b"quoted-printable":
            raise MultipartUnsupported("quoted-printable part")
        # the part's data: up to the first NL + dash followed by a terminator
        end = _data_end(body, i, dash, nl)
        if end is None:
            # partReader: io.ErrUnexpectedEOF (io.ReadAll / io.Copy error)
            res["error"] = "unexpected EOF"
            return res
        data = body[i:end]
        i = end
        disp, dparams = _disposition(hdr)
        name = dparams.get(b"name", b"") if disp == b"form-data" else b""
        for k in sorted(set(k for k, _ in hdr)):
            for kk, v in hdr:
                if kk == k:
                    res["part_headers"].append((name, k + b": " + v))
        filename = dparams.get(b"filename", b"")
        if filename:
            total += len(data)
            res["files"].append((b"", filename))
            fs = res["files_sizes"]
            for x, (k, _) in enumerate(fs):
                if k.lower() == filename.lower():
                    fs[x] = (k, str(len(data)).encode())
                    break
            else:
                fs.append((filename, str(len(data)).encode()))
            res["files_names"].append((b"", name))
        else:
            total += len(data)
            res["args_post"].append((name, data))
        res["combined_size"] = str(total).encode()


def _is_final(line: bytes, dash: bytes, nl: bytes) -> bool:
    if not line.startswith(dash + b"--"):
        return False
    rest = line[len(dash) + 2:].lstrip(b" \t")
    return rest == b"" or rest == nl


def _data_end(body: bytes, i: int, dash: bytes, nl: bytes) -> Optional[int]:
    """End of the part data starting at body[i] (scanUntilBoundary)."""
    n = len(body)

    def after_ok(k: int) -> bool:  # matchAfterPrefix(...) == +1 at body[k]
        if k >= n:
            return True
        c = body[k]
        if c in b" \t\r\n":
            return True
        return c == ord("-") and k + 1 < n and body[k + 1] == ord("-")

    if body.startswith(dash, i) and after_ok(i + len(dash)):
        return i
    pat = nl + dash
    k = body.find(pat, i)
    while k >= 0:
        if after_ok(k + len(pat)):
            return k
        k = body.find(pat, k + 1)
    return None
