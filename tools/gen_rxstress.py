"""Generate the CRS-scale regex stress rules (rulesets/rxstress.conf) and the
C2X ruleset (rulesets/crs_pl1_rxstress.conf = crs_pl1.conf + rxstress.conf).

CRS v4's 942 / 932 / 941 detection regexes are assembled by the CRS
toolchain from word lists into trie-factored alternations of several KB each
(`(?i)\\b(?:a(?:dd(?:dat|tim)e|es_(?:de|en)crypt|...)|b(?:enchmark|...)...)\\s*\\(`).
CRS itself is a download (reference Makefile:185-206); this script writes 20
rules of that shape from seeded synthetic vocabularies, 2-6 KB of pattern
text each, so the DFA state cap / NFA fallback is exercised at C2 scale:

* 8 x 942-style: `(?i)` keyword trie + a call / operator context;
* 6 x 932-style: command-separator prefix + command trie + argument context;
* 4 x 941-style: tag / event-handler trie + attribute context;
* 2 x wide-context rules (a trie followed by a counted gap and a second trie)
  whose DFAs exceed the state cap and run as NFA position tables.

Each rule reads ARGS / ARGS_NAMES / REQUEST_COOKIES(_NAMES) with CRS's
transformation chains and adds to the PL1 anomaly score, ids 942900+.
`words()` is shared with traffic generation (`traffic.rxstress_payloads`).

    python tools/gen_rxstress.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED942

SYL = ["al", "be", "ca", "de", "ex", "fo", "ge", "hi", "in", "jo", "ka", "lo", "ma", "ne", "or", "pe", "qu", "ra",
       "se", "to", "un", "ve", "wa", "xi", "yo", "ze", "str", "cat", "sel", "upd", "del", "ins", "ch", "sh", "th",
       "_to_", "_", "2", "32", "64"]
SQL_STEMS = ["select", "union", "insert", "update", "delete", "drop", "alter", "create", "exec", "execute", "declare",
             "cast", "convert", "concat", "substr", "substring", "ascii", "char", "chr", "hex", "unhex", "sleep",
             "benchmark", "waitfor", "delay", "load_file", "outfile", "dumpfile", "information_schema", "sysobjects",
             "xp_cmdshell", "sp_executesql", "pg_sleep", "dbms_pipe", "utl_http", "extractvalue", "updatexml",
             "group_concat", "json_extract", "having", "order", "group", "limit", "offset", "procedure", "analyse"]
CMD_STEMS = ["cat", "tac", "nl", "head", "tail", "more", "less", "curl", "wget", "nc", "ncat", "netcat", "bash", "sh",
             "zsh", "ksh", "dash", "python", "perl", "ruby", "php", "lua", "awk", "sed", "find", "xargs", "chmod",
             "chown", "base64", "xxd", "od", "openssl", "socat", "telnet", "ssh", "scp", "rsync", "tftp", "ftp",
             "crontab", "nohup", "setsid", "busybox", "env", "eval", "exec", "printf", "echo", "id", "whoami", "uname"]
XSS_STEMS = ["onload", "onerror", "onclick", "onmouseover", "onfocus", "onblur", "onchange", "onsubmit", "onkeydown",
             "onkeyup", "onanimationstart", "ontransitionend", "onpointerdown", "ontoggle", "onbegin", "script",
             "iframe", "object", "embed", "applet", "svg", "math", "style", "link", "meta", "base", "form", "input",
             "button", "details", "marquee", "video", "audio", "source", "template", "frameset", "isindex"]


def words(kind: str, n: int, seed: int, stems: bool = True):
    """n distinct lowercase words of the family: real stems (unless stems is
    False) plus seeded syllable compounds around them (deterministic)."""
    rng = np.random.default_rng(seed)
    with_stems = stems
    stems = {"sql": SQL_STEMS, "cmd": CMD_STEMS, "xss": XSS_STEMS}[kind]
    out = []
    seen = set(stems)
    if with_stems:
        out += list(stems)
    while len(out) < n:
        k = int(rng.integers(0, 3))
        stem = stems[int(rng.integers(0, len(stems)))]
        parts = [SYL[int(rng.integers(0, len(SYL)))] for _ in range(int(rng.integers(1, 4)))]
        if k == 0:
            w = stem + "".join(parts)
        elif k == 1:
            w = "".join(parts) + stem
        else:
            w = "".join(parts[:1]) + stem + "".join(parts[1:])
        w = w.strip("_")
        if 3 <= len(w) <= 18 and w not in seen:
            seen.add(w)
            out.append(w)
    return out[:n]


def _esc(c: str) -> str:
    return "\\" + c if c in ".^$*+?()[]{}|\\/" else c


def trie_regex(ws):
    """Trie-factored alternation of ws (regexp-assemble style)."""
    trie = {}
    for w in ws:
        t = trie
        for c in w:
            t = t.setdefault(c, {})
        t[""] = {}

    def emit(t):
        end = "" in t
        keys = sorted(k for k in t if k)
        alts = []
        for k in keys:
            sub = t[k]
            # collapse single-child chains
            s = _esc(k)
            while len(sub) == 1 and "" not in sub:
                (k2, sub2), = sub.items()
                s += _esc(k2)
                sub = sub2
            rest = emit(sub) if (len(sub) > 1 or "" not in sub) else ""
            alts.append(s + rest)
        if not alts:
            return ""
        body = alts[0] if len(alts) == 1 and not end else "(?:" + "|".join(alts) + ")"
        if end:
            body = ("(?:" + "|".join(alts) + ")?") if len(alts) > 1 else (body + "?" if len(alts[0]) == 1 else "(?:" + alts[0] + ")?")
        return body

    return emit(trie)


def sized_words(kind, seed, lo_bytes, hi_bytes, stems=True):
    """a word list whose trie regex lands in [lo_bytes, hi_bytes]"""
    target = (lo_bytes + hi_bytes) // 2
    n = 64
    while True:
        ws = words(kind, n, seed, stems)
        size = len(trie_regex(ws))
        if size >= lo_bytes or n > 4000:
            break
        n = int(n * max(1.1, target / max(size, 1)))
    while len(trie_regex(ws)) > hi_bytes and len(ws) > 16:
        ws = ws[: int(len(ws) * 0.9)]
    return ws


SEP = r"(?:^|[;&|`\n]|\$\(|\|\|)"
A = "ARGS|ARGS_NAMES|REQUEST_COOKIES|!REQUEST_COOKIES:/__utm/|REQUEST_COOKIES_NAMES"
T_SQL = "t:none,t:urlDecodeUni,t:lowercase"
T_CMD = "t:none,t:cmdLine"
T_XSS = "t:none,t:utf8toUnicode,t:urlDecodeUni,t:htmlEntityDecode,t:jsDecode,t:cssDecode,t:removeNulls"


def rules():
    """(id, family, regex, transformations, msg, tag, score variable, word lists, context index)"""
    out = []
    rid = 942900
    sizes = [(2000, 3000), (3000, 4500), (4500, 6000)]
    for i in range(8):  # 942-style
        lo, hi = sizes[i % 3]
        ws = sized_words("sql", SEED + i, lo, hi)
        ctx = [r"[\s\x0b]*?\(", r"[\s\x0b]+(?:all|distinct|from|into|where)\b", r"[\s\x0b]*?[=<>!]+[\s\x0b]*?[0-9'\"]",
               r"\b"][i % 4]
        out.append((rid, "sql", "(?i)\\b" + trie_regex(ws) + ctx, T_SQL, "SQL Injection Attack (assembled keyword set %d)" % i,
                    "attack-sqli", "sql_injection_score", (ws,), i % 4))
        rid += 1
    for i in range(6):  # 932-style
        lo, hi = sizes[(i + 1) % 3]
        ws = sized_words("cmd", SEED + 100 + i, lo, hi)
        ctx = [r"(?:[\s<>&|),;]|$)", r"[\s\x0b]+[^\s\x0b]", r"\b"][i % 3]
        out.append((rid, "cmd", SEP + r"[\s\x0b]*" + trie_regex(ws) + ctx, T_CMD,
                    "Remote Command Execution: Unix Command Injection (assembled command set %d)" % i, "attack-rce",
                    "rce_score", (ws,), i % 3))
        rid += 1
    for i in range(4):  # 941-style
        lo, hi = sizes[(i + 2) % 3]
        ws = sized_words("xss", SEED + 200 + i, lo, hi)
        ctx = [r"[\s\x0b]*=", r"[\s\x0b/>]", r"[^a-z]", r"[\s\x0b]*=[\s\x0b]*['\"]?"][i % 4]
        pre = ["<", r"[\s\x0b\"'`;/0-9=]", "<", r"[\s\x0b\"'`;/]"][i % 4]
        out.append((rid, "xss", "(?i)" + pre + trie_regex(ws) + ctx, T_XSS,
                    "XSS Filter - Category %d: assembled tag / handler set" % i, "attack-xss", "xss_score", (ws,), i % 4))
        rid += 1
    for i in range(2):  # wide context: beyond the DFA state cap -> NFA position tables
        ws1 = sized_words("sql", SEED + 300 + i, 1200, 1800, stems=False)
        ws2 = words("sql", 40, SEED + 400 + i, stems=False)
        out.append((rid, "wide", "(?i)" + trie_regex(ws1) + r"[^\n]{0,%d}?" % (24 + 8 * i) + trie_regex(ws2) + r"\b",
                    T_SQL, "SQL Injection Attack (keyword pair within a window %d)" % i, "attack-sqli",
                    "sql_injection_score", (ws1, ws2), 24 + 8 * i))
        rid += 1
    return out


def conf_text():
    lines = ["# CRS-scale regex stress rules (tools/gen_rxstress.py; seeded, assembled-trie shape of CRS v4",
             "# 942 / 932 / 941).  Added to crs_pl1.conf as rulesets/crs_pl1_rxstress.conf (bench --config c2x).", ""]
    for rid, fam, rx, tr, msg, tag, score, _, _ in rules():
        rx_q = rx.replace('"', '\\"')  # SecLang keeps backslashes; only the quote is escaped
        lines.append(
            'SecRule %s "@rx %s" "id:%d,phase:2,block,capture,%s,msg:\'%s\',tag:\'%s\',tag:\'paranoia-level/1\','
            "ver:'OWASP_CRS/4.23.0',severity:'CRITICAL',setvar:'tx.%s=+%%{tx.critical_anomaly_score}',"
            "setvar:'tx.inbound_anomaly_score_pl1=+%%{tx.critical_anomaly_score}'\"" % (A, rx_q, rid, tr, msg, tag, score))
    return "\n".join(lines) + "\n"


def payloads(n: int = 64, seed: int = SEED):
    """n attack-shaped strings, cycling over the stress rules, each built to
    hit its rule (a word of the rule's list in the rule's context) -- or, for
    every third one, a near miss (the word without its context)."""
    rng = np.random.default_rng(seed ^ 0xABC)
    rs = rules()
    out = []
    for k in range(n):
        rid, fam, _, _, _, _, _, lists, ctx = rs[k % len(rs)]
        w = lists[0][int(rng.integers(0, len(lists[0])))]
        miss = k % 3 == 2
        if fam == "sql":
            tail = ["(1)", " from t", " = '1", " x"][ctx]
            out.append(("1 " + w + ("" if miss else tail)).encode())
        elif fam == "cmd":
            tail = [" /etc/hosts", " -la", ".sh"][ctx]
            out.append(("x" + ("" if miss else "|") + w + tail).encode())
        elif fam == "xss":
            pre = ["<", " ", "<", " "][ctx]
            tail = [" =alert(1)", "/", ">", "='x'"][ctx]
            out.append(((pre if not miss else "") + w + tail).encode())
        else:
            w2 = lists[1][int(rng.integers(0, len(lists[1])))]
            gap = "y" * (ctx + (8 if miss else -4))
            out.append((w + gap + " " + w2).encode())
    return out


def main():
    text = conf_text()
    sizes = [len(r[2]) for r in rules()]
    open(os.path.join(ROOT, "rulesets", "rxstress.conf"), "w").write(text)
    base = open(os.path.join(ROOT, "rulesets", "crs_pl1.conf")).read()
    # after the last detection file, before the blocking evaluation (949110),
    # outside every paranoia-gated region, so their scores count at PL1
    marker = "SecMarker \"END-REQUEST-944-APPLICATION-ATTACK-JAVA\"\n"
    if marker not in base:
        sys.exit("marker not found in crs_pl1.conf: %s" % marker)
    i = base.index(marker) + len(marker)
    open(os.path.join(ROOT, "rulesets", "crs_pl1_rxstress.conf"), "w").write(base[:i] + text + "\n" + base[i:])
    print("rules %d, pattern bytes %d (min %d, max %d)" % (len(sizes), sum(sizes), min(sizes), max(sizes)))


if __name__ == "__main__":
    main()
