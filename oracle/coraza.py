"""CPU oracle: Coraza v3.3.3 rule evaluation restated in Python.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import this module, and only as the
checker.  The product (the HIP engine behind `include/gpuinspect.h`) never
routes through it.

Reference anchors
-----------------
* The operator compiles each ConfigMap's SecLang with
  `coraza.NewWAF(coraza.NewWAFConfig().WithDirectives(data))`
  (/root/reference/internal/controller/ruleset_controller.go:158-171) and
  joins the ConfigMaps with "\\n" (:173-176) before `Cache.Put` (:180-181).
* The evaluation itself happens in the data plane (coraza-proxy-wasm,
  config/samples/engine.yaml:12) running coraza/v3 v3.3.3 (go.mod:6).
  That module is NOT vendored under /root/reference and no Go toolchain is
  present, so every function below marked [upstream] restates the published
  algorithm of the named coraza source file from knowledge of that module.
  See DESIGN.md "Oracle" for the list of semantic choices that are
  therefore "parity unpinned" beyond the reference's own KATs.
* The KATs that *are* pinned come from the reference's tests:
  test/integration/coreruleset_test.go:57-127, reconcile_test.go:43-88,
  multiple_gateways_test.go:89-100, multi_engine_gateway_test.go:82-138,
  test/framework/resources.go:122-127 (SimpleBlockRule) and
  config/samples/README.md:36-60.  They live in tests/golden/kats.json.

Evaluation model (mirrors coraza's Transaction):
  ProcessURI -> AddRequestHeader* -> ProcessRequestHeaders (phase 1)
  -> ProcessRequestBody (body processor, phase 2) -> MatchedRules/Interruption.
"""

from __future__ import annotations

import posixpath
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import goregex, libinjection, multipart, xmlbody

# ---------------------------------------------------------------------------
# Errors
# ---------------------------------------------------------------------------


class SecLangError(ValueError):
    """A directive that coraza.NewWAF would reject (ruleset_controller.go:160)."""


class SecLangUnsupported(SecLangError):
    """SecLang coraza.NewWAF accepts whose request-phase evaluation this
    oracle (and the engine, GI_EUNSUPPORTED) does not model: a phase 1-2 rule
    reading a response variable, or using an operator / transformation / ctl
    of the response path.  The same constructs in phase 3-5 rules are fine:
    the request path never evaluates those phases."""


# ---------------------------------------------------------------------------
# Variables (coraza internal/variables) -- name -> (kind, case_insensitive)
# kind: 'single' | 'map' | 'names' | 'args' | 'argnames' | 'tx' | 'matched'
# ---------------------------------------------------------------------------

SINGLE_VARS = {
    "REQUEST_METHOD", "REQUEST_PROTOCOL", "REQUEST_URI", "REQUEST_URI_RAW",
    "REQUEST_LINE", "REQUEST_FILENAME", "REQUEST_BASENAME", "QUERY_STRING",
    "REQUEST_BODY", "REQUEST_BODY_LENGTH", "REQBODY_ERROR", "REQBODY_ERROR_MSG",
    "REQBODY_PROCESSOR", "MULTIPART_STRICT_ERROR", "ARGS_COMBINED_SIZE",
    "FULL_REQUEST_LENGTH", "MATCHED_VAR", "MATCHED_VAR_NAME",
    "REMOTE_ADDR", "REMOTE_PORT", "SERVER_NAME", "URLENCODED_ERROR",
    "FILES_COMBINED_SIZE", "INBOUND_DATA_ERROR",
}
# FULL_REQUEST_LENGTH and URLENCODED_ERROR are declared variables that
# coraza v3.3.3's transaction never sets [upstream internal/corazawaf/
# transaction.go; bodyprocessors/urlencoded.go]: they read "" (parity unpinned).
MAP_VARS = {
    # name: (source collection(s), case_insensitive_keys)
    "ARGS_GET": (("ARGS_GET",), False),
    "ARGS_POST": (("ARGS_POST",), False),
    "ARGS": (("ARGS_GET", "ARGS_POST"), False),
    "REQUEST_HEADERS": (("REQUEST_HEADERS",), True),
    "REQUEST_COOKIES": (("REQUEST_COOKIES",), False),
    "TX": (("TX",), True),
    "MATCHED_VARS": (("MATCHED_VARS",), True),
    # the XML body processor's values (oracle/xmlbody.py): keys "//@*" and "/*"
    "XML": (("XML",), False),
    # multipart collections (oracle/multipart.py); keys: "" for FILES /
    # FILES_NAMES, the file name for FILES_SIZES, the part name for
    # MULTIPART_PART_HEADERS (coraza collections.NewMap: case-insensitive)
    "FILES": (("FILES",), True),
    "FILES_NAMES": (("FILES_NAMES",), True),
    "FILES_SIZES": (("FILES_SIZES",), True),
    "FILES_TMPNAMES": (("FILES_TMPNAMES",), True),
    "MULTIPART_PART_HEADERS": (("MULTIPART_PART_HEADERS",), True),
}
NAMES_VARS = {
    "ARGS_GET_NAMES": (("ARGS_GET",), False),
    "ARGS_POST_NAMES": (("ARGS_POST",), False),
    "ARGS_NAMES": (("ARGS_GET", "ARGS_POST"), False),
    "REQUEST_HEADERS_NAMES": (("REQUEST_HEADERS",), True),
    "REQUEST_COOKIES_NAMES": (("REQUEST_COOKIES",), False),
    "MATCHED_VARS_NAMES": (("MATCHED_VARS",), True),
}
# [upstream internal/variables/variables.go]: declared variables the request
# path does not evaluate (the response phases', and a few without a value here)
DEFERRED_VARS = {
    "RESPONSE_BODY", "RESPONSE_STATUS", "RESPONSE_HEADERS", "RESPONSE_HEADERS_NAMES", "RESPONSE_PROTOCOL",
    "RESPONSE_CONTENT_TYPE", "RESPONSE_CONTENT_LENGTH", "RESPONSE_ARGS", "RESPONSE_XML", "RES_BODY_PROCESSOR",
    "OUTBOUND_DATA_ERROR", "STATUS_LINE", "SERVER_ADDR", "SERVER_PORT", "UNIQUE_ID", "REMOTE_HOST",
    "HIGHEST_SEVERITY", "DURATION", "REQBODY_PROCESSOR_ERROR", "REQBODY_PROCESSOR_ERROR_MSG", "ARGS_PATH",
    "FILES_TMP_CONTENT", "MULTIPART_FILENAME", "MULTIPART_NAME", "MULTIPART_DATA_AFTER", "GEO", "RULE", "JSON",
    "ENV", "REQUEST_XML", "AUTH_TYPE", "TIME", "TIME_DAY", "TIME_EPOCH", "TIME_HOUR", "TIME_MIN", "TIME_MON",
    "TIME_SEC", "TIME_WDAY", "TIME_YEAR",
}
ALL_VARS = SINGLE_VARS | set(MAP_VARS) | set(NAMES_VARS) | DEFERRED_VARS
# operators / transformations coraza v3.3.3 has that are not modelled here
DEFERRED_OPERATORS = {"geolookup", "inspectfile", "pmfromdataset", "ipmatchfromdataset", "rbl", "restpath",
                      "strmatch", "validatenid", "validateschema", "verifycc", "verifycpf", "verifyssn",
                      "fuzzyhash"}
DEFERRED_TRANSFORMS = {"removecomments", "sqlhexdecode", "uppercase"}
# [upstream internal/actions/ctl.go]: evaluated / without effect on a request-phase verdict
CTL_EVALUATED = {"ruleremovebyid", "ruleremovetargetbyid", "ruleremovebytag", "ruleremovetargetbytag",
                 "ruleremovebymsg", "ruleremovetargetbymsg", "ruleengine", "requestbodyprocessor",
                 "requestbodyaccess", "forcerequestbodyvariable"}
CTL_NO_EFFECT = {"auditengine", "auditlogparts", "debugloglevel", "responsebodyaccess", "responsebodylimit",
                 "responsebodyprocessor", "forceresponsebodyvariable", "hashengine", "hashenforcement"}


@dataclass
class RuleVariable:
    name: str
    key: str = ""              # literal key ("" = whole collection)
    key_rx: Optional[goregex.GoRegexp] = None
    count: bool = False
    exceptions: List[Tuple[str, Optional[goregex.GoRegexp]]] = field(default_factory=list)


@dataclass
class Operator:
    name: str
    arg: str
    negate: bool
    rx: Optional[goregex.GoRegexp] = None
    phrases: Optional[List[bytes]] = None
    byte_ok: Optional[List[bool]] = None
    macro: Optional[list] = None
    nets: Optional[list] = None  # @ipMatch networks (ipmatch_networks)


@dataclass
class SetVar:
    key: list              # macro template for the key (after "tx.")
    value: Optional[list]  # macro template; None for "!tx.x" (remove)
    remove: bool = False


@dataclass
class Rule:
    id: int = 0
    phase: int = 2
    line: int = 0
    variables: List[RuleVariable] = field(default_factory=list)
    op: Optional[Operator] = None
    transforms: List[str] = field(default_factory=list)
    disruptive: str = ""          # "" | deny | drop | pass | block | redirect | allow
    status: int = 0
    capture: bool = False
    multimatch: bool = False
    setvars: List[SetVar] = field(default_factory=list)
    ctls: List[Tuple[str, str]] = field(default_factory=list)
    nondisruptive_order: List[Tuple[str, object]] = field(default_factory=list)
    skip: int = 0
    skip_after: str = ""
    secmark: str = ""
    chain: Optional["Rule"] = None
    parent_id: int = 0
    has_chain_action: bool = False
    tags: List[str] = field(default_factory=list)
    msg: str = ""
    deferred: str = ""   # a construct of the response path (SecLangUnsupported in phases 1-2)


@dataclass
class WafConfig:
    rule_engine: str = "On"       # On | Off | DetectionOnly
    request_body_access: bool = False
    request_body_limit: int = 134217728
    request_body_limit_action: str = "Reject"
    args_limit: int = 1000        # SecArgumentsLimit (WAF.ArgumentLimit)
    rules: List[Rule] = field(default_factory=list)
    default_actions: Dict[int, str] = field(default_factory=dict)


# ---------------------------------------------------------------------------
# SecLang parser  [upstream internal/seclang/{parser,directives,rule_parser}.go]
# ---------------------------------------------------------------------------

IGNORED_DIRECTIVES = {
    "secresponsebodyaccess", "secresponsebodymimetype", "secresponsebodylimit",
    "secresponsebodylimitaction", "secauditengine", "secauditlogtype",
    "secauditlog", "secauditlogformat", "secauditlogparts",
    "secauditlogrelevantstatus", "secauditlogstoragedir", "secauditlogdirmode",
    "secauditlogfilemode", "secdebuglog", "secdebuglogLevel".lower(),
    "seccomponentsignature", "secrequestbodyinmemorylimit", "sectmpdir",
    "secdatadir", "secargumentseparator", "seccollectiontimeout",
    "secrequestbodynofileslimit", "secuploaddir", "secuploadkeepfiles",
    "secuploadfilemode", "secunicodemap", "secpcrematchlimit",
    "secpcrematchlimitrecursion", "secstatusengine", "secconnengine",
    "secserversignature", "sechttpblkey", "secwebappid", "secsensorid",
    "secrequestbodyjsondepthlimit", "secmarker_", "secresponsebodymimetypesclear", "seccookieformat",
    "secuploadfilelimit", "secignorerulecompilationerrors",
}

ACTION_TYPES = {
    # disruptive
    "deny": "disruptive", "drop": "disruptive", "pass": "disruptive",
    "block": "disruptive", "redirect": "disruptive", "allow": "disruptive",
    # flow
    "chain": "flow", "skip": "flow", "skipafter": "flow",
    # metadata
    "id": "metadata", "phase": "metadata", "msg": "metadata", "tag": "metadata",
    "severity": "metadata", "ver": "metadata", "rev": "metadata",
    "maturity": "metadata", "accuracy": "metadata",
    # data
    "status": "data", "xmlns": "data",
    # non-disruptive
    "t": "nondisruptive", "setvar": "nondisruptive", "capture": "nondisruptive",
    "log": "nondisruptive", "nolog": "nondisruptive", "auditlog": "nondisruptive",
    "noauditlog": "nondisruptive", "logdata": "nondisruptive",
    "multimatch": "nondisruptive", "ctl": "nondisruptive",
    "expirevar": "nondisruptive", "initcol": "nondisruptive",
    "sanitisearg": "nondisruptive", "sanitisematched": "nondisruptive",
    "setenv": "nondisruptive", "append": "nondisruptive",
    "sanitiserequestheader": "nondisruptive", "sanitiseresponseheader": "nondisruptive",
}

PHASE_NAMES = {"request": 2, "response": 4, "logging": 5}


_ASCII_WS = " \t\r\n\v\f"


def _split_lines(text: str):
    """parser.go parseString: trim each line, join '\\' continuations."""
    buf = ""
    lineno = 0
    start = 0
    for raw in text.split("\n"):
        lineno += 1
        line = raw.strip(_ASCII_WS)
        if not buf:
            start = lineno
        if line.endswith("\\"):
            buf += line[:-1]
        else:
            buf += line
            yield start, buf
            buf = ""
    if buf:
        yield start, buf


def _cut_quoted(s: str):
    """rule_parser.go cutQuotedString: escapes are kept, \\" does not end it."""
    if not s or s[0] != '"':
        raise SecLangError("expected quoted string: %r" % s)
    for i in range(1, len(s)):
        if s[i] != '"':
            continue
        if s[i - 1] == "\\":
            continue
        return s[1:i], s[i + 1:]
    raise SecLangError("expected terminating quote: %r" % s)


def _parse_actions_list(s: str):
    """Split `a,b:'x,y',c:d` into [(key, value)] (quotes stripped)."""
    out = []
    cur = ""
    quote = False
    for ch in s:
        if ch == "'":
            quote = not quote
            cur += ch
            continue
        if ch == "," and not quote:
            out.append(cur)
            cur = ""
            continue
        cur += ch
    if cur.strip():
        out.append(cur)
    res = []
    for item in out:
        item = item.strip()
        if not item:
            continue
        if ":" in item:
            k, v = item.split(":", 1)
        else:
            k, v = item, ""
        k = k.strip().lower()
        v = v.strip()
        if len(v) >= 2 and v[0] == "'" and v[-1] == "'":
            v = v[1:-1]
        if k not in ACTION_TYPES:
            raise SecLangError("unknown action %r" % k)
        res.append((k, v))
    return res


def _parse_variables(s: str, rule: Rule):
    parts = []
    cur = ""
    in_rx = False
    i = 0
    while i < len(s):
        ch = s[i]
        if ch == "/" and cur.endswith(":") and not in_rx:
            in_rx = True
            cur += ch
        elif ch == "/" and in_rx:
            in_rx = False
            cur += ch
        elif ch == "|" and not in_rx:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
        i += 1
    parts.append(cur)
    for p in parts:
        p = p.strip()
        if not p:
            continue
        neg = cnt = False
        if p[0] == "!":
            neg = True
            p = p[1:]
        elif p[0] == "&":
            cnt = True
            p = p[1:]
        name, _, key = p.partition(":")
        name = name.upper()
        if name not in ALL_VARS:
            raise SecLangError("unknown variable %r" % name)
        if name in DEFERRED_VARS and not rule.deferred:
            rule.deferred = "unsupported variable " + name
        key_rx = None
        if len(key) >= 2 and key[0] == "'" and key[-1] == "'":
            key = key[1:-1]
        if len(key) > 2 and key[0] == "/" and key[-1] == "/":
            try:
                key_rx = goregex.compile_go(key[1:-1])
            except goregex.RegexError as e:
                raise SecLangError("invalid key regex %r: %s" % (key, e))
            key = key[1:-1]
        if neg:
            # rule.go AddVariableNegation: applies to earlier vars of same type
            matched = False
            for rv in rule.variables:
                if rv.name == name:
                    rv.exceptions.append((key.lower(), key_rx))
                    matched = True
            if not matched:
                raise SecLangError("cannot negate variable %s that is not targeted" % name)
            continue
        if name in SINGLE_VARS and key:
            raise SecLangError("variable %s does not accept a key" % name)
        rule.variables.append(RuleVariable(name=name, key=key if key_rx is None else "",
                                           key_rx=key_rx, count=cnt))


# macro templates [upstream internal/macro]: list of str | ("var", NAME, key)
_MACRO_RE = re.compile(r"%\{([^}]+)\}")


def parse_macro(s: str):
    parts = []
    pos = 0
    for m in _MACRO_RE.finditer(s):
        if m.start() > pos:
            parts.append(s[pos:m.start()])
        ref = m.group(1)
        name, _, key = ref.partition(".")
        parts.append(("var", name.upper(), key.lower()))
        pos = m.end()
    if pos < len(s):
        parts.append(s[pos:])
    return parts


def _has_macro(parts):
    return any(isinstance(p, tuple) for p in parts)


def pm_file_phrases(data: bytes):
    """coraza internal/operators/pm_from_file.go: bufio.Scanner lines (a
    trailing '\\r' dropped), strings.TrimSpace, skip empty lines and '#'
    comments, strings.ToLower (ASCII here, like the @pm matcher's folding)."""
    out = []
    for line in data.split(b"\n"):
        if line.endswith(b"\r"):
            line = line[:-1]
        line = line.strip(b" \t\n\v\f\r")
        if not line or line[:1] == b"#":
            continue
        out.append(line.lower())
    return out


def _parse_operator(opstr: str, data_files=None, rule=None) -> Operator:
    # rule_parser.go ParseOperator: default operator is @rx
    if len(opstr) == 0 or (opstr[0] != "@" and (len(opstr) < 2 or opstr[1] != "@")):
        opstr = "@rx " + opstr
    raw, _, data = opstr.partition(" ")
    raw = raw.strip()
    data = data.strip()
    negate = False
    if raw.startswith("!@"):
        negate = True
        name = raw[2:]
    elif raw.startswith("@"):
        name = raw[1:]
    else:
        name = raw
    name_l = name.lower()
    op = Operator(name=name_l, arg=data, negate=negate)
    if name_l == "rx":
        try:
            op.rx = goregex.rx_compile(data)
        except goregex.RegexError as e:
            raise SecLangError("invalid regex %r: %s" % (data, e))
    elif name_l == "pm":
        op.phrases = [p.encode().lower() for p in data.lower().split(" ") if p]
    elif name_l == "pmfromfile":
        if data_files is None or data not in data_files:
            raise SecLangError("open %s: no such file or directory" % data)
        op.phrases = pm_file_phrases(data_files[data])
    elif name_l in ("contains", "streq", "beginswith", "endswith", "within",
                    "eq", "ge", "gt", "le", "lt", "containsword"):
        op.macro = parse_macro(data)
    elif name_l == "validatebyterange":
        ok = [False] * 256
        for part in data.split(","):
            part = part.strip()
            if not part:
                continue
            if "-" in part:
                a, b = part.split("-", 1)
                a, b = int(a), int(b)
                if not (0 <= a <= 255 and 0 <= b <= 255 and a <= b):
                    raise SecLangError("invalid byte range %r" % part)
                for x in range(a, b + 1):
                    ok[x] = True
            else:
                a = int(part)
                if not 0 <= a <= 255:
                    raise SecLangError("invalid byte %r" % part)
                ok[a] = True
        op.byte_ok = ok
    elif name_l in ("unconditionalmatch", "nomatch", "validateurlencoding",
                    "validateutf8encoding", "detectsqli", "detectxss"):
        pass
    elif name_l == "ipmatch":
        op.nets = ipmatch_networks(data)
    elif name_l in ("ipmatchfromfile", "ipmatchf"):
        # ipmatchfromfile.go: one network per line, '#' comments and blanks skipped
        if data_files is None or data not in data_files:
            raise SecLangError("open %s: no such file or directory" % data)
        lines = []
        for line in data_files[data].split(b"\n"):
            line = line.rstrip(b"\r").strip()
            if line and line[:1] != b"#":
                lines.append(line.decode("latin-1"))
        op.name = "ipmatch"
        op.nets = ipmatch_networks(",".join(lines))
    elif name_l in DEFERRED_OPERATORS:
        if rule is not None and not rule.deferred:
            rule.deferred = "unsupported operator @" + name
    else:
        raise SecLangError("invalid operator @%s" % name)
    return op


TRANSFORMS_SUPPORTED = {
    "none", "lowercase", "urldecode", "urldecodeuni", "htmlentitydecode",
    "removenulls", "replacenulls", "removewhitespace", "compresswhitespace",
    "replacecomments", "cmdline", "length", "trim", "trimleft", "trimright",
    "normalizepath", "normalisepath", "normalizepathwin", "normalisepathwin",
    "jsdecode", "utf8tounicode", "base64decode", "base64decodeext", "base64encode", "hexdecode",
    "hexencode", "sha1", "md5", "urlencode", "cssdecode", "escapeseqdecode", "removecommentschar",
}


def _apply_actions(rule: Rule, actions, is_child: bool):
    for k, v in actions:
        if k == "id":
            rule.id = int(v)
        elif k == "phase":
            vl = v.lower()
            rule.phase = PHASE_NAMES[vl] if vl in PHASE_NAMES else int(v)
        elif k in ("deny", "drop", "pass", "block", "redirect", "allow"):
            rule.disruptive = k
            if k == "allow":
                # [upstream internal/actions/allow.go Init]
                a = v.lower()
                if a in ("phase", "request"):
                    rule.disruptive = "allow:" + a
                elif a:
                    raise SecLangError("invalid argument %s for allow" % v)
        elif k == "status":
            rule.status = int(v)
        elif k == "chain":
            rule.has_chain_action = True
        elif k == "skip":
            rule.skip = int(v)
        elif k == "skipafter":
            rule.skip_after = v
        elif k == "t":
            tl = v.lower()
            if tl == "none":
                rule.transforms = []
            else:
                if tl in DEFERRED_TRANSFORMS:
                    if not rule.deferred:
                        rule.deferred = "unsupported transformation t:" + v
                    continue
                if tl not in TRANSFORMS_SUPPORTED:
                    raise SecLangError("invalid transformation t:%s" % v)
                rule.transforms.append(tl)
        elif k == "capture":
            rule.capture = True
        elif k == "multimatch":
            rule.multimatch = True
        elif k == "tag":
            rule.tags.append(v)
        elif k == "msg":
            rule.msg = v
        elif k == "setvar":
            sv = _parse_setvar(v)
            rule.setvars.append(sv)
            rule.nondisruptive_order.append(("setvar", sv))
        elif k == "ctl":
            name, _, val = v.partition("=")
            name = name.strip()
            cl = (name.lower(), val.strip())
            if cl[0] in CTL_NO_EFFECT:
                continue
            if cl[0] == "requestbodylimit":
                if not rule.deferred:
                    rule.deferred = "unsupported ctl requestbodylimit"
                continue
            if cl[0] not in CTL_EVALUATED:
                raise SecLangError("unknown ctl %s" % name)
            rule.ctls.append(cl)
            rule.nondisruptive_order.append(("ctl", cl))


def _parse_setvar(v: str) -> SetVar:
    # [upstream internal/actions/setvar.go] "tx.key=value", "!tx.key"
    remove = False
    if v.startswith("!"):
        remove = True
        v = v[1:]
    col, _, rest = v.partition(".")
    if col.strip().lower() != "tx":
        raise SecLangError("setvar only supports the TX collection")
    if remove:
        return SetVar(key=parse_macro(rest.strip()), value=None, remove=True)
    key, eq, value = rest.partition("=")
    if not eq:
        value = ""
    return SetVar(key=parse_macro(key.strip()), value=parse_macro(value))


def merge_default_actions(actions, defaults):
    """[upstream rule_parser.go mergeActions]: default non-metadata,
    non-disruptive actions are prepended; the default disruptive action is
    appended only when the rule uses `block`."""
    res = []
    da = None
    for k, v in defaults:
        t = ACTION_TYPES[k]
        if t == "disruptive":
            da = (k, v)
            continue
        if t == "metadata":
            continue
        res.append((k, v))
    has_block = False
    for k, v in actions:
        if k == "block":
            has_block = True
        res.append((k, v))
    if has_block and da is not None:
        res.append(da)
    return res


def _id_range(s: str):
    """An id or "lo-hi" (directives.go / ctl.go rangeToInts) -> (lo, hi)."""
    a, dash, b = s[1:].partition("-") if s[:1] == "-" else s.partition("-")
    if s[:1] == "-":
        a = "-" + a
    lo, ok = go_atoi(a.encode())
    if not ok:
        raise SecLangError("invalid id %s" % s)
    if not dash:
        return lo, lo
    hi, ok = go_atoi(b.encode())
    if not ok:
        raise SecLangError("invalid id %s" % s)
    return lo, hi


def parse_seclang(text: str, data_files=None) -> WafConfig:
    cfg = WafConfig()
    pending_parent: Optional[Rule] = None
    chain_tail: Optional[Rule] = None
    ids = {}  # top-level rule id -> count (RuleGroup.Add rejects a repeated non-zero id)

    def strip_q(x):
        return x.strip().strip('"')

    def remove(pred):
        kept = []
        for r in cfg.rules:
            if pred(r):
                if r.id:
                    ids[r.id] -= 1
                    if not ids[r.id]:
                        del ids[r.id]
            else:
                kept.append(r)
        cfg.rules = kept
    for lineno, line in _split_lines(text):
        if not line or line[0] == "#":
            continue
        directive, _, opts = line.partition(" ")
        if len(opts) >= 3 and opts[0] == '"' and opts[-1] == '"':
            opts = opts.strip('"')
        d = directive.lower()
        if d == "secruleengine":
            o = opts.strip().lower()
            cfg.rule_engine = {"on": "On", "off": "Off", "detectiononly": "DetectionOnly"}[o]
        elif d == "secrequestbodyaccess":
            cfg.request_body_access = opts.strip().lower() == "on"
        elif d == "secrequestbodylimit":
            cfg.request_body_limit = int(opts.strip())
        elif d == "secrequestbodylimitaction":
            cfg.request_body_limit_action = opts.strip()
        elif d == "secargumentslimit":
            v, ok = go_atoi(opts.strip().encode())
            if not ok:
                raise SecLangError("syntax error: SecArgumentsLimit [POSITIVE_INT]")
            cfg.args_limit = v
        elif d in ("secruleremovebyid", "secruleremovebytag", "secruleremovebymsg"):
            # [upstream internal/seclang/directives.go directiveSecRuleRemoveBy*]
            if pending_parent is not None:
                raise SecLangError("%s inside a chain" % directive)
            if not opts.strip():
                raise SecLangError("expected options for %s" % directive)
            if d == "secruleremovebyid":
                for part in opts.split():
                    lo, hi = _id_range(part)
                    remove(lambda r: lo <= r.id <= hi)
            elif d == "secruleremovebytag":
                tag = strip_q(opts)
                remove(lambda r: tag in r.tags)
            else:
                msg = strip_q(opts)
                remove(lambda r: not r.secmark and r.msg == msg)
        elif d in ("secruleupdatetargetbyid", "secruleupdatetargetbytag", "secruleupdatetargetbymsg",
                   "secruleupdateactionbyid"):
            # [upstream directives.go directiveSecRuleUpdate{Target,Action}By*]
            if pending_parent is not None:
                raise SecLangError("%s inside a chain" % directive)
            sel, sp, arg = opts.strip().partition(" ")
            if not sp:
                raise SecLangError("syntax error: %s" % directive)
            sel, arg = strip_q(sel), strip_q(arg)
            by_id = d in ("secruleupdatetargetbyid", "secruleupdateactionbyid")
            lo, hi = _id_range(sel) if by_id else (0, -1)
            hit = [r for r in cfg.rules if not r.secmark and (
                (lo <= r.id <= hi) if by_id else (sel in r.tags if d.endswith("bytag") else r.msg == sel))]
            if by_id and lo == hi and not hit:
                raise SecLangError('%s: rule "%s" not found' % (directive, sel))
            for r in hit:
                if d == "secruleupdateactionbyid":
                    acts = _parse_actions_list(arg)
                    for k, _ in acts:
                        if k in ("id", "chain"):
                            raise SecLangError("SecRuleUpdateActionById: action %s cannot be updated" % k)
                    if any(ACTION_TYPES[k] == "disruptive" for k, _ in acts):
                        r.disruptive = ""  # [upstream] Rule.ClearDisruptiveActions
                    _apply_actions(r, acts, False)
                    c = r.chain
                    while c is not None:
                        c.phase = r.phase
                        c = c.chain
                else:
                    _parse_variables(arg, r)
        elif d == "secdefaultaction":
            acts = _parse_actions_list(opts)
            phase = 2
            for k, v in acts:
                if k == "phase":
                    vl = v.lower()
                    phase = PHASE_NAMES[vl] if vl in PHASE_NAMES else int(v)
            cfg.default_actions[phase] = acts
        elif d == "secmarker":
            r = Rule(id=0, phase=0, line=lineno, secmark=opts.strip().strip('"'))
            if pending_parent is not None:
                raise SecLangError("SecMarker inside a chain")
            cfg.rules.append(r)
        elif d in ("secrule", "secaction"):
            rule = Rule(line=lineno)
            if d == "secrule":
                rest = opts.lstrip()
                if rest.startswith('"'):
                    vars_s, rest = _cut_quoted(rest)
                else:
                    vars_s, _, rest = rest.partition(" ")
                _parse_variables(vars_s, rule)
                rest = rest.strip()
                opstr, rest = _cut_quoted(rest)
                rule.op = _parse_operator(opstr, data_files, rule)
                rest = rest.strip()
                acts_s = rest.strip('"') if rest else ""
            else:
                acts_s = opts
            actions = _parse_actions_list(acts_s) if acts_s else []
            is_child = pending_parent is not None
            if not is_child:
                phase = 2
                for k, v in actions:
                    if k == "phase":
                        vl = v.lower()
                        phase = PHASE_NAMES[vl] if vl in PHASE_NAMES else int(v)
                defaults = cfg.default_actions.get(phase)
                if defaults:
                    actions = merge_default_actions(actions, defaults)
            _apply_actions(rule, actions, is_child)
            if is_child:
                rule.parent_id = pending_parent.id
                rule.phase = pending_parent.phase
                chain_tail.chain = rule
                chain_tail = rule
                if not rule.has_chain_action:
                    pending_parent = None
                    chain_tail = None
            else:
                if rule.id == 0:
                    raise SecLangError("rule id is required (line %d)" % lineno)
                if rule.id in ids:
                    raise SecLangError("there is a another rule with id %d" % rule.id)
                ids[rule.id] = 1
                cfg.rules.append(rule)
                if rule.has_chain_action:
                    pending_parent = rule
                    chain_tail = rule
        elif d in IGNORED_DIRECTIVES or d.startswith("secaudit") or d.startswith("secdebug"):
            pass
        else:
            raise SecLangError("unknown directive %r" % directive)
    if pending_parent is not None:
        raise SecLangError("unterminated chain")
    # phases 3-5 are never evaluated by the request path: their response-side
    # constructs are accepted there, and rejected in a phase 1-2 rule
    for r in cfg.rules:
        if r.phase not in (1, 2):
            continue
        c = r
        while c is not None:
            if c.deferred:
                raise SecLangUnsupported("%s (rule %d, phase %d)" % (c.deferred, r.id, r.phase))
            c = c.chain
    return cfg


# ---------------------------------------------------------------------------
# Transformations  [upstream internal/transformations/*.go, ModSecurity ports]
# All operate on bytes.
# ---------------------------------------------------------------------------

_HEX = b"0123456789abcdefABCDEF"


def _ishex(c: int) -> bool:
    return (48 <= c <= 57) or (65 <= c <= 70) or (97 <= c <= 102)


def _x2c(a: int, b: int) -> int:
    return int(bytes([a, b]), 16)


def t_lowercase(d: bytes) -> bytes:
    # Go strings.ToLower: ASCII fast path, else strings.Map(unicode.ToLower)
    if d.isascii():
        return d.lower()
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        c = d[i]
        if c < 0x80:
            out.append(c + 32 if 65 <= c <= 90 else c)
            i += 1
            continue
        r, w = goregex._decode_rune(d, i)
        if r == 0xFFFD and w == 1:
            out += "�".encode()
        else:
            out += chr(go_to_lower(r)).encode()
        i += w
    return bytes(out)


def go_to_lower(r: int) -> int:
    """unicode.ToLower (simple mapping)."""
    if r == 0x130:
        return 0x69
    lo = chr(r).lower()
    return ord(lo) if len(lo) == 1 else r


def t_urldecode(d: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        c = d[i]
        if c == 0x25:
            if i + 2 < n and _ishex(d[i + 1]) and _ishex(d[i + 2]):
                out.append(_x2c(d[i + 1], d[i + 2]))
                i += 3
            else:
                out.append(c)
                i += 1
        else:
            out.append(0x20 if c == 0x2B else c)
            i += 1
    return bytes(out)


def t_urldecodeuni(d: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        c = d[i]
        if c == 0x25:
            if i + 1 < n and d[i + 1] in (0x75, 0x55):  # %u
                if i + 5 < n:
                    if all(_ishex(d[i + k]) for k in range(2, 6)):
                        b = _x2c(d[i + 4], d[i + 5])
                        if 0 < b < 0x5F and d[i + 2] in (0x66, 0x46) and d[i + 3] in (0x66, 0x46):
                            b += 0x20
                        out.append(b)
                        i += 6
                    else:
                        out += d[i:i + 2]
                        i += 2
                else:
                    out += d[i:i + 2]
                    i += 2
            else:
                if i + 2 < n and _ishex(d[i + 1]) and _ishex(d[i + 2]):
                    out.append(_x2c(d[i + 1], d[i + 2]))
                    i += 3
                else:
                    out.append(c)
                    i += 1
        else:
            out.append(0x20 if c == 0x2B else c)
            i += 1
    return bytes(out)


def _isalnum(c):
    return 48 <= c <= 57 or 65 <= c <= 90 or 97 <= c <= 122


def _strtol_byte(digits: bytes, base: int) -> int:
    v = int(digits, base)
    if v > 0x7FFFFFFFFFFFFFFF:  # strtol/ParseInt saturate on overflow
        v = 0x7FFFFFFFFFFFFFFF
    return v & 0xFF


def t_htmlentitydecode(d: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        copy = 1
        if d[i] == 0x26 and i + 1 < n:  # '&'
            j = i + 1
            if d[j] == 0x23:  # '#'
                copy += 1
                if j + 1 < n:
                    j += 1
                    if d[j] in (0x78, 0x58):  # x X
                        copy += 1
                        if j + 1 < n:
                            j += 1
                            k = j
                            while j < n and _ishex(d[j]):
                                j += 1
                            if j > k:
                                out.append(_strtol_byte(d[k:j], 16))
                                i = j + 1 if (j < n and d[j] == 0x3B) else j
                                continue
                    else:
                        k = j
                        while j < n and 48 <= d[j] <= 57:
                            j += 1
                        if j > k:
                            out.append(_strtol_byte(d[k:j], 10))
                            i = j + 1 if (j < n and d[j] == 0x3B) else j
                            continue
            else:
                k = j
                while j < n and _isalnum(d[j]):
                    j += 1
                if j > k:
                    name = d[k:j].lower()
                    ent = {b"quot": 0x22, b"amp": 0x26, b"lt": 0x3C, b"gt": 0x3E, b"nbsp": 0xA0}.get(name)
                    if ent is not None:
                        out.append(ent)
                        i = j + 1 if (j < n and d[j] == 0x3B) else j
                        continue
                    copy = j - k + 1
        z = 0
        while z < copy and i < n:
            out.append(d[i])
            i += 1
            z += 1
    return bytes(out)


_WS = {0x20, 0x09, 0x0A, 0x0B, 0x0C, 0x0D}


def t_removewhitespace(d: bytes) -> bytes:
    return bytes(c for c in d if c not in _WS and c != 0xA0)


def t_compresswhitespace(d: bytes) -> bytes:
    out = bytearray()
    inws = False
    for c in d:
        if c in _WS or c == 0xA0:
            if not inws:
                out.append(0x20)
            inws = True
        else:
            inws = False
            out.append(c)
    return bytes(out)


def t_replacecomments(d: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(d)
    inc = False
    while i < n:
        if not inc:
            if d[i] == 0x2F and i + 1 < n and d[i + 1] == 0x2A:
                inc = True
                i += 2
            else:
                out.append(d[i])
                i += 1
        else:
            if d[i] == 0x2A and i + 1 < n and d[i + 1] == 0x2F:
                inc = False
                i += 2
                out.append(0x20)
            else:
                i += 1
    if inc:
        out.append(0x20)
    return bytes(out)


def t_cmdline(d: bytes) -> bytes:
    out = bytearray()
    space = False
    for c in d:
        if c in (0x22, 0x27, 0x5C, 0x5E):
            continue
        if c in (0x20, 0x2C, 0x3B, 0x09, 0x0D, 0x0A):
            if not space:
                out.append(0x20)
                space = True
            continue
        if c in (0x2F, 0x28):
            if space:
                out.pop()
                space = False
            out.append(c)
            continue
        out.append(c + 32 if 65 <= c <= 90 else c)
        space = False
    return bytes(out)


_GO_SPACE = {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029,
             0x202F, 0x205F, 0x3000} | set(range(0x2000, 0x200B))


def _trim_left(d: bytes) -> bytes:
    i = 0
    while i < len(d):
        r, w = goregex._decode_rune(d, i)
        if r == 0xFFFD and w == 1:
            break
        if r not in _GO_SPACE:
            break
        i += w
    return d[i:]


def _trim_right(d: bytes) -> bytes:
    end = len(d)
    while end > 0:
        # find start of last rune (Go DecodeLastRune)
        s = end - 1
        while s > 0 and end - s < 4 and 0x80 <= d[s] <= 0xBF:
            s -= 1
        r, w = goregex._decode_rune(d, s)
        if s + w != end:
            r, w = 0xFFFD, 1
            s = end - 1
        if r not in _GO_SPACE or (r == 0xFFFD):
            break
        end = s
    return d[:end]


def t_normalizepath(d: bytes, win: bool = False) -> bytes:
    if win:
        d = d.replace(b"\\", b"/")
    if len(d) < 1:
        return d
    clean = _go_path_clean(d)
    if clean == b".":
        return b""
    if d[-1:] == b"/":
        return clean + b"/"
    return clean


def _go_path_clean(p: bytes) -> bytes:
    """Go path.Clean."""
    if p == b"":
        return b"."
    rooted = p[:1] == b"/"
    n = len(p)
    out = bytearray()
    r, dotdot = 0, 0
    if rooted:
        out.append(0x2F)
        r, dotdot = 1, 1
    while r < n:
        if p[r] == 0x2F:
            r += 1
        elif p[r] == 0x2E and (r + 1 == n or p[r + 1] == 0x2F):
            r += 1
        elif p[r] == 0x2E and p[r + 1] == 0x2E and (r + 2 == n or p[r + 2] == 0x2F):
            r += 2
            if len(out) > dotdot:
                w = len(out) - 1
                while w > dotdot and out[w] != 0x2F:
                    w -= 1
                del out[w:]
            elif not rooted:
                if len(out) > 0:
                    out.append(0x2F)
                out += b".."
                dotdot = len(out)
        else:
            if (rooted and len(out) != 1) or (not rooted and len(out) != 0):
                out.append(0x2F)
            while r < n and p[r] != 0x2F:
                out.append(p[r])
                r += 1
    if len(out) == 0:
        return b"."
    return bytes(out)


def _isodigit(c):
    return 48 <= c <= 55


def t_jsdecode(d: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        if d[i] == 0x5C:
            if i + 5 < n and d[i + 1] == 0x75 and all(_ishex(d[i + k]) for k in range(2, 6)):
                b = _x2c(d[i + 4], d[i + 5])
                if 0 < b < 0x5F and d[i + 2] in (0x66, 0x46) and d[i + 3] in (0x66, 0x46):
                    b += 0x20
                out.append(b)
                i += 6
            elif i + 3 < n and d[i + 1] == 0x78 and _ishex(d[i + 2]) and _ishex(d[i + 3]):
                out.append(_x2c(d[i + 2], d[i + 3]))
                i += 4
            elif i + 1 < n and _isodigit(d[i + 1]):
                j = 0
                buf = bytearray()
                while i + 1 + j < n and j < 3:
                    buf.append(d[i + 1 + j])
                    j += 1
                    if not (i + 1 + j < n and _isodigit(d[i + 1 + j])):
                        break
                if j == 3 and buf[0] > 0x33:
                    j = 2
                    buf = buf[:2]
                out.append(int(bytes(buf), 8) & 0xFF)
                i += 1 + j
            elif i + 1 < n:
                c = d[i + 1]
                c = {0x61: 7, 0x62: 8, 0x66: 12, 0x6E: 10, 0x72: 13, 0x74: 9, 0x76: 11}.get(c, c)
                out.append(c)
                i += 2
            else:
                out += d[i:]
                i = n
        else:
            out.append(d[i])
            i += 1
    return bytes(out)


def t_utf8tounicode(d: bytes) -> bytes:
    """ModSecurity utf8_unicode_inplace_ex restated: every valid multi-byte
    UTF-8 sequence becomes %uXXXX (lowercase hex, >= 4 digits); ASCII and
    invalid bytes are copied.  [upstream utf8toUnicode.go, unverified]"""
    if all(c < 0x80 for c in d):
        return d
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        c = d[i]
        if c < 0x80:
            out.append(c)
            i += 1
            continue
        r, w = goregex._decode_rune(d, i)
        if r == 0xFFFD and w == 1:
            out.append(c)
            i += 1
            continue
        out += b"%u" + (b"%04x" % r)
        i += w
    return bytes(out)


_B64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
_B64_REV = {c: i for i, c in enumerate(_B64)}


def t_base64decode(d: bytes) -> bytes:
    """[upstream base64decode.go] forgiving decode: CR/LF skipped; stops at
    '=', ' ', a byte > 127 or any other byte outside the alphabet; a trailing
    2 / 3 symbol group yields 1 / 2 bytes, a lone symbol nothing."""
    out = bytearray()
    x = n = 0
    for c in d:
        if c in (0x0D, 0x0A):
            continue
        v = _B64_REV.get(c)
        if v is None:
            break
        x = (x << 6) | v
        n += 1
        if n == 4:
            out += bytes([(x >> 16) & 0xFF, (x >> 8) & 0xFF, x & 0xFF])
            x = n = 0
    if n == 2:
        out.append((x << 12 >> 16) & 0xFF)
    elif n == 3:
        x <<= 6
        out += bytes([(x >> 16) & 0xFF, (x >> 8) & 0xFF])
    return bytes(out)


def t_base64decodeext(d: bytes) -> bytes:
    """ModSecurity decode_base64_ext restated [upstream base64decodeext.go]:
    bytes outside the alphabet (padding included) are skipped, every other
    symbol decoded; a partial trailing byte is dropped."""
    out = bytearray()
    x = n = 0
    for c in d:
        v = _B64_REV.get(c)
        if v is None:
            continue
        x = (x << 6) | v
        n += 1
        if n == 4:
            out += bytes([(x >> 16) & 0xFF, (x >> 8) & 0xFF, x & 0xFF])
            x = n = 0
    if n == 2:
        out.append((x << 12 >> 16) & 0xFF)
    elif n == 3:
        x <<= 6
        out += bytes([(x >> 16) & 0xFF, (x >> 8) & 0xFF])
    return bytes(out)


def t_base64encode(d: bytes) -> bytes:
    """Go base64.StdEncoding.EncodeToString."""
    import base64
    return base64.b64encode(d)


def t_hexdecode(d: bytes) -> bytes:
    """Go hex.DecodeString; on an error (odd length, a non-hex byte) the
    transformation fails and rule.go executeTransformations keeps the value."""
    if len(d) % 2 or not all(_ishex(c) for c in d):
        return d
    return bytes.fromhex(d.decode())


def t_hexencode(d: bytes) -> bytes:
    return d.hex().encode()


def t_sha1(d: bytes) -> bytes:
    import hashlib
    return hashlib.sha1(d).digest()


def t_md5(d: bytes) -> bytes:
    import hashlib
    return hashlib.md5(d).digest()


def t_urlencode(d: bytes) -> bytes:
    """ModSecurity url_encode [upstream urlencode.go]: ' ' -> '+'; '*', digits
    and letters kept; every other byte %xx (lowercase hex)."""
    out = bytearray()
    for c in d:
        if c == 0x20:
            out.append(0x2B)
        elif c == 0x2A or 48 <= c <= 57 or 65 <= c <= 90 or 97 <= c <= 122:
            out.append(c)
        else:
            out += b"%%%02x" % c
    return bytes(out)


def _cisspace(c: int) -> bool:
    return c == 0x20 or 9 <= c <= 13


def t_cssdecode(d: bytes) -> bytes:
    """ModSecurity css_decode_inplace [upstream cssdecode.go]: a backslash and
    1-6 hex digits -> one byte (the last two digits; full-width ff01-ff5e +0x20
    for 4 digits, for 5 / 6 digits only with leading zeros), one whitespace
    after the escape eaten; backslash-newline removed; any other escaped byte
    kept; a trailing backslash dropped."""
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        if d[i] != 0x5C:
            out.append(d[i])
            i += 1
            continue
        if i + 1 >= n:
            i += 1
            continue
        i += 1
        j = 0
        while j < 6 and i + j < n and _ishex(d[i + j]):
            j += 1
        if j == 0:
            if d[i] == 0x0A:
                i += 1
            else:
                out.append(d[i])
                i += 1
            continue
        if j == 1:
            out.append(int(d[i:i + 1], 16))
        else:
            v = _x2c(d[i + j - 2], d[i + j - 1])
            full = j == 4 or (j == 5 and d[i] == 0x30) or (j == 6 and d[i] == 0x30 and d[i + 1] == 0x30)
            if full and 0 < v < 0x5F and d[i + j - 3] in (0x66, 0x46) and d[i + j - 4] in (0x66, 0x46):
                v += 0x20
            out.append(v)
        if i + j < n and _cisspace(d[i + j]):
            j += 1
        i += j
    return bytes(out)


_ESC_SIMPLE = {0x61: 7, 0x62: 8, 0x66: 12, 0x6E: 10, 0x72: 13, 0x74: 9, 0x76: 11, 0x5C: 0x5C, 0x3F: 0x3F,
               0x27: 0x27, 0x22: 0x22}


def t_escapeseqdecode(d: bytes) -> bytes:
    """ModSecurity ansi_c_sequences_decode_inplace [upstream escapeseqdecode.go]:
    \\a \\b \\f \\n \\r \\t \\v \\\\ \\? \\' \\"; \\xHH (two hex digits);
    \\ooo (1-3 octal digits, value & 0xFF); an unrecognised escape keeps only
    the escaped byte; a trailing backslash is kept."""
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        if d[i] != 0x5C or i + 1 >= n:
            out.append(d[i])
            i += 1
            continue
        e = d[i + 1]
        if e in _ESC_SIMPLE:
            out.append(_ESC_SIMPLE[e])
            i += 2
            continue
        if e in (0x78, 0x58):
            if i + 3 < n and _ishex(d[i + 2]) and _ishex(d[i + 3]):
                out.append(_x2c(d[i + 2], d[i + 3]))
                i += 4
                continue
        elif _isodigit(e):
            j = 0
            while i + 1 + j < n and j < 3:
                j += 1
                if not (i + 1 + j < n and _isodigit(d[i + 1 + j])):
                    break
            out.append(int(d[i + 1:i + 1 + j], 8) & 0xFF)
            i += 1 + j
            continue
        out.append(e)
        i += 2
    return bytes(out)


def t_removecommentschar(d: bytes) -> bytes:
    """ModSecurity remove_comments_char [upstream removecommentschar.go]: drops
    the comment markers /* */ <!-- --> -- and #."""
    out = bytearray()
    i, n = 0, len(d)
    while i < n:
        if d.startswith(b"/*", i) or d.startswith(b"*/", i):
            i += 2
        elif d.startswith(b"<!--", i):
            i += 4
        elif d.startswith(b"-->", i):
            i += 3
        elif d.startswith(b"--", i):
            i += 2
        elif d[i] == 0x23:
            i += 1
        else:
            out.append(d[i])
            i += 1
    return bytes(out)


TRANSFORM_FNS = {
    "utf8tounicode": t_utf8tounicode,
    "lowercase": t_lowercase,
    "urldecode": t_urldecode,
    "urldecodeuni": t_urldecodeuni,
    "htmlentitydecode": t_htmlentitydecode,
    "removenulls": lambda d: d.replace(b"\x00", b""),
    "replacenulls": lambda d: d.replace(b"\x00", b" "),
    "removewhitespace": t_removewhitespace,
    "compresswhitespace": t_compresswhitespace,
    "replacecomments": t_replacecomments,
    "cmdline": t_cmdline,
    "length": lambda d: str(len(d)).encode(),
    "trim": lambda d: _trim_right(_trim_left(d)),
    "trimleft": _trim_left,
    "trimright": _trim_right,
    "normalizepath": t_normalizepath,
    "normalisepath": t_normalizepath,
    "normalizepathwin": lambda d: t_normalizepath(d, True),
    "normalisepathwin": lambda d: t_normalizepath(d, True),
    "jsdecode": t_jsdecode,
    "base64decode": t_base64decode,
    "base64decodeext": t_base64decodeext,
    "base64encode": t_base64encode,
    "hexdecode": t_hexdecode,
    "hexencode": t_hexencode,
    "sha1": t_sha1,
    "md5": t_md5,
    "urlencode": t_urlencode,
    "cssdecode": t_cssdecode,
    "escapeseqdecode": t_escapeseqdecode,
    "removecommentschar": t_removecommentschar,
}


# ---------------------------------------------------------------------------
# Request model, URI parsing  [upstream corazawaf/transaction.go ProcessURI,
# Go net/url Parse/String, coraza internal/url ParseQuery]
# ---------------------------------------------------------------------------


@dataclass
class Request:
    method: bytes
    uri: bytes
    proto: bytes = b"HTTP/1.1"
    headers: List[Tuple[bytes, bytes]] = field(default_factory=list)
    body: bytes = b""
    remote_addr: bytes = b""   # ProcessConnection client -> REMOTE_ADDR
    remote_port: int = 0       # -> REMOTE_PORT (strconv.Itoa)
    server_name: bytes = b""   # SetServerName -> SERVER_NAME


class UnsupportedInput(ValueError):
    """Input outside the engine's supported subset (flagged, not guessed)."""


def query_unescape(s: bytes) -> bytes:
    """Lenient %XX / '+' decoding (invalid escapes kept verbatim)."""
    out = bytearray()
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c == 0x25 and i + 2 < n and _ishex(s[i + 1]) and _ishex(s[i + 2]):
            out.append(_x2c(s[i + 1], s[i + 2]))
            i += 3
        elif c == 0x2B:
            out.append(0x20)
            i += 1
        else:
            out.append(c)
            i += 1
    return bytes(out)


def parse_query(q: bytes, sep: int = 0x26):
    """[upstream internal/url ParseQuery] -> list of (key, value) in order."""
    out = []
    while q:
        i = q.find(bytes([sep]))
        if i >= 0:
            key, q = q[:i], q[i + 1:]
        else:
            key, q = q, b""
        if key == b"":
            continue
        value = b""
        j = key.find(b"=")
        if j >= 0:
            key, value = key[:j], key[j + 1:]
        out.append((query_unescape(key), query_unescape(value)))
    return out


def _go_should_escape_path(c: int) -> bool:
    if 65 <= c <= 90 or 97 <= c <= 122 or 48 <= c <= 57:
        return False
    if c in b"-_.~":
        return False
    if c in b"$&+,/:;=?@":
        return c == 0x3F
    return True


def _go_escape_path(s: bytes) -> bytes:
    out = bytearray()
    for c in s:
        if _go_should_escape_path(c):
            out += b"%" + ("%02X" % c).encode()
        else:
            out.append(c)
    return bytes(out)


def _go_valid_encoded_path(s: bytes) -> bool:
    for c in s:
        if c in b"!$&'()*+,;=:@[]%":
            continue
        if _go_should_escape_path(c):
            return False
    return True


def _go_unescape_path(s: bytes):
    """net/url unescape(s, encodePath): strict; returns None on bad escape."""
    out = bytearray()
    i, n = 0, len(s)
    while i < n:
        if s[i] == 0x25:
            if i + 2 >= n or not _ishex(s[i + 1]) or not _ishex(s[i + 2]):
                return None
            out.append(_x2c(s[i + 1], s[i + 2]))
            i += 3
        else:
            out.append(s[i])
            i += 1
    return bytes(out)


class _GoURLError(ValueError):
    """net/url.Parse returned an error."""


def _go_should_escape(c: int, mode: str) -> bool:
    """net/url shouldEscape for the modes ProcessURI's url.Parse / String use:
    "path", "host", "user" (encodePath, encodeHost, encodeUserPassword)."""
    if 65 <= c <= 90 or 97 <= c <= 122 or 48 <= c <= 57:
        return False
    if mode == "host" and c in b"!$&'()*+,;=:[]<>\"":
        return False
    if c in b"-_.~":
        return False
    if c in b"$&+,/:;=?@":
        if mode == "user":
            return c in b"@/?:"
        if mode == "path":
            return c == 0x3F
    return True


def _go_escape(s: bytes, mode: str) -> bytes:
    out = bytearray()
    for c in s:
        if _go_should_escape(c, mode):
            out += b"%" + ("%02X" % c).encode()
        else:
            out.append(c)
    return bytes(out)


def _go_unescape(s: bytes, mode: str) -> bytes:
    """net/url unescape (strict: a malformed escape is an error; in a host,
    %-escapes only for non-ASCII bytes or %25, and no ASCII byte that must be
    escaped)."""
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c == 0x25:
            if i + 2 >= n or not _ishex(s[i + 1]) or not _ishex(s[i + 2]):
                raise _GoURLError("invalid URL escape")
            if mode == "host" and int(chr(s[i + 1]), 16) < 8 and s[i:i + 3] != b"%25":
                raise _GoURLError("invalid URL escape")
            i += 3
        else:
            if mode == "host" and c < 0x80 and _go_should_escape(c, "host"):
                raise _GoURLError("invalid character in host name")
            i += 1
    out = bytearray()
    i = 0
    while i < n:
        if s[i] == 0x25:
            out.append(_x2c(s[i + 1], s[i + 2]))
            i += 3
        else:
            out.append(s[i])
            i += 1
    return bytes(out)


def _go_valid_port(p: bytes) -> bool:
    if p == b"":
        return True
    return p[:1] == b":" and all(0x30 <= c <= 0x39 for c in p[1:])


def _go_parse_host(h: bytes) -> bytes:
    if h.startswith(b"["):
        i = h.rfind(b"]")
        if i < 0:
            raise _GoURLError("missing ']' in host")
        if not _go_valid_port(h[i + 1:]):
            raise _GoURLError("invalid port")
        if h[:i].find(b"%25") >= 0:
            # RFC 6874 zone identifiers: not restated (the GPU flags them the same way)
            raise UnsupportedInput("IPv6 zone in the request-target host")
    else:
        i = h.rfind(b":")
        if i >= 0 and not _go_valid_port(h[i:]):
            raise _GoURLError("invalid port")
    return _go_unescape(h, "host")


_USER_OK = b"-._:~!$&'()*+,;=%@"


def _go_parse_authority(a: bytes):
    """-> (userinfo string as URL.String() writes it, or None; host)."""
    i = a.rfind(b"@")
    host = _go_parse_host(a if i < 0 else a[i + 1:])
    if i < 0:
        return None, host
    ui = a[:i]
    for c in ui:
        if not (65 <= c <= 90 or 97 <= c <= 122 or 48 <= c <= 57 or c in _USER_OK):
            raise _GoURLError("invalid userinfo")
    if b":" not in ui:
        return _go_escape(_go_unescape(ui, "user"), "user"), host
    u, _, pw = ui.partition(b":")
    return _go_escape(_go_unescape(u, "user"), "user") + b":" + _go_escape(_go_unescape(pw, "user"), "user"), host


def _go_url_parse(u: bytes):
    """[Go net/url] Parse(u) (no fragment: ProcessURI cut it) and String():
    -> (String(), Path, RawQuery).  Raises _GoURLError where Parse fails."""
    if u == b"*":
        return b"*", b"*", b""
    scheme, rest = b"", u
    for i, c in enumerate(u):  # getScheme
        if 65 <= c <= 90 or 97 <= c <= 122:
            continue
        if 48 <= c <= 57 or c in b"+-.":
            if i == 0:
                break
            continue
        if c == 0x3A:
            if i == 0:
                raise _GoURLError("missing protocol scheme")
            scheme, rest = u[:i].lower(), u[i + 1:]
        break
    force_q = rest.endswith(b"?") and rest.count(b"?") == 1
    if force_q:
        rest, query = rest[:-1], b""
    else:
        rest, _, query = rest.partition(b"?")
    tail = b"?" + query if (force_q or query) else b""
    if not rest.startswith(b"/"):
        if scheme:  # rootless: opaque
            return scheme + b":" + rest + tail, b"", query
        if b":" in rest.split(b"/", 1)[0]:
            raise _GoURLError("first path segment in URL cannot contain colon")
    user, host, omit_host = None, b"", False
    if (scheme or not rest.startswith(b"///")) and rest.startswith(b"//"):
        auth, rest = rest[2:], b""
        j = auth.find(b"/")
        if j >= 0:
            auth, rest = auth[:j], auth[j:]
        user, host = _go_parse_authority(auth)
    elif scheme and rest.startswith(b"/"):
        omit_host = True
    path = _go_unescape(rest, "path")
    # EscapedPath: the raw path when it is a valid encoding of Path
    if _go_escape_path(path) == rest or _go_valid_encoded_path(rest):
        esc = rest
    else:
        esc = _go_escape_path(path)
    out = b""
    if scheme:
        out += scheme + b":"
    if scheme or host or user is not None:
        if not (omit_host and host == b"" and user is None):
            if host or path or user is not None:
                out += b"//"
            if user is not None:
                out += user + b"@"
            if host:
                out += _go_escape(host, "host")
    if esc and esc[:1] != b"/" and host:
        out += b"/"
    if out == b"" and b":" in esc.split(b"/", 1)[0]:
        out += b"./"
    return out + esc + tail, path, query


def process_uri(uri: bytes):
    """[upstream corazawaf/transaction.go ProcessURI]: REQUEST_URI_RAW, then
    url.Parse of the '#'-stripped target -> REQUEST_URI = URL.String(),
    REQUEST_FILENAME = URL.Path, QUERY_STRING = URL.RawQuery, ARGS_GET; when
    url.Parse fails, REQUEST_URI / REQUEST_FILENAME are the target itself and
    there are no GET args.  Returns (dict of the URI variables, ARGS_GET).

    Every request-target form Parse accepts: origin ("/p?q"), absolute
    ("http://user@h:80/p"), scheme-relative ("//h/p"), asterisk, opaque
    ("mailto:x"), relative ("p/q").  Only an IPv6 zone identifier
    ("[fe80::1%25en0]") raises UnsupportedInput (flagged the same way on the GPU).
    """
    v = {"REQUEST_URI_RAW": uri}
    u = uri
    h = u.find(b"#")
    if h >= 0:
        u = u[:h]
    args = []
    try:
        if any(c < 0x20 or c == 0x7F for c in u):
            raise _GoURLError("invalid control character in URL")
        s_, path, query = _go_url_parse(u)
        v["REQUEST_URI"] = s_
        args = parse_query(query)
    except _GoURLError:
        v["REQUEST_URI"] = u
        path, query = u, b""
    v["REQUEST_FILENAME"] = path
    v["QUERY_STRING"] = query
    off = path.rfind(b"/")
    if off != -1 and len(path) > off + 1:
        v["REQUEST_BASENAME"] = path[off + 1:]
    else:
        v["REQUEST_BASENAME"] = path
    return v, args


def parse_cookies(value: bytes):
    """[upstream] cookie header parsing: split ';', trim, cut '='."""
    out = []
    raw = value.strip(b" \t\r\n\v\f")
    while raw:
        part, sep, raw = raw.partition(b";")
        part = part.strip(b" \t\r\n\v\f")
        if not part:
            continue
        name, _, val = part.partition(b"=")
        out.append((name, val))
    return out


# ---------------------------------------------------------------------------
# Transaction + rule evaluation  [upstream corazawaf/{transaction,rulegroup,rule}.go]
# ---------------------------------------------------------------------------


JSON_MAX_DEPTH = 64  # engine limit (gjson itself recurses without one): deeper -> UnsupportedInput


def JSON_FLAT_LIMIT(n: int) -> int:
    """Engine limit on flattened JSON bytes (kernels.hip parse_json_body)."""
    return 4 * n + 1024
_JSON_WS = b" \t\n\r"
_JSON_SIMPLE_ESC = {0x22: 0x22, 0x5C: 0x5C, 0x2F: 0x2F, 0x62: 0x08, 0x66: 0x0C, 0x6E: 0x0A, 0x72: 0x0D, 0x74: 0x09}


def _utf8(r: int) -> bytes:
    """Go utf8.EncodeRune (surrogates and out-of-range -> U+FFFD)."""
    if 0xD800 <= r <= 0xDFFF or r > 0x10FFFF:
        r = 0xFFFD
    return chr(r).encode("utf-8")


def _json_unescape(raw: bytes) -> bytes:
    """[upstream tidwall/gjson v1.18.0 unescape] on a validated string body.

    A \\uXXXX in the surrogate range consumes a directly following \\uXXXX
    and decodes the pair with utf16.DecodeRune (U+FFFD unless high+low);
    a lone surrogate encodes as U+FFFD."""
    out = bytearray()
    i, n = 0, len(raw)
    while i < n:
        c = raw[i]
        if c != 0x5C:
            out.append(c)
            i += 1
            continue
        e = raw[i + 1]
        if e != 0x75:
            out.append(_JSON_SIMPLE_ESC[e])
            i += 2
            continue
        r = int(raw[i + 2:i + 6], 16)
        i += 6
        if 0xD800 <= r < 0xE000:
            if n - i >= 6 and raw[i] == 0x5C and raw[i + 1] == 0x75:
                r2 = int(raw[i + 2:i + 6], 16)
                i += 6
                if 0xD800 <= r < 0xDC00 and 0xDC00 <= r2 < 0xE000:
                    r = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00)
                else:
                    r = 0xFFFD
            else:
                r = 0xFFFD
        out += _utf8(r)
    return bytes(out)


class _JsonInvalid(Exception):
    pass


class _JsonReader:
    """RFC 8259 recursive-descent reader (the grammar gjson.Valid accepts)."""

    def __init__(self, s: bytes):
        self.s = s
        self.i = 0

    def ws(self):
        s, i = self.s, self.i
        while i < len(s) and s[i] in _JSON_WS:
            i += 1
        self.i = i

    def peek(self) -> int:
        if self.i >= len(self.s):
            raise _JsonInvalid()
        return self.s[self.i]

    def expect(self, c: int):
        if self.peek() != c:
            raise _JsonInvalid()
        self.i += 1

    def string(self) -> bytes:
        """Returns the unescaped contents of the string at self.i (sets
        self.escaped)."""
        self.expect(0x22)
        s, start = self.s, self.i
        i, esc = start, False
        while True:
            if i >= len(s):
                raise _JsonInvalid()
            c = s[i]
            if c == 0x22:
                break
            if c < 0x20:
                raise _JsonInvalid()
            if c == 0x5C:
                esc = True
                if i + 1 >= len(s):
                    raise _JsonInvalid()
                e = s[i + 1]
                if e == 0x75:
                    h = s[i + 2:i + 6]
                    if len(h) != 4 or not all(_ishex(x) for x in h):
                        raise _JsonInvalid()
                    i += 6
                    continue
                if e not in _JSON_SIMPLE_ESC:
                    raise _JsonInvalid()
                i += 2
                continue
            i += 1
        self.i = i + 1
        raw = s[start:i]
        self.escaped = esc
        return _json_unescape(raw) if esc else raw

    def number(self) -> bytes:
        s, start = self.s, self.i
        m = re.compile(rb"-?(?:0|[1-9][0-9]*)(?:\.[0-9]+)?(?:[eE][+-]?[0-9]+)?").match(s, start)
        if m is None or m.end() == start:
            raise _JsonInvalid()
        self.i = m.end()
        return s[start:self.i]


class JsonBodyError(ValueError):
    """The body is not JSON (gjson.Valid false): [upstream json.go readJSON]
    returns an error, ProcessRequestBody calls generateRequestBodyError and
    still evaluates phase 2 (REQBODY_ERROR=1, no ARGS_POST)."""


def json_flatten(body: bytes):
    """[upstream coraza internal/bodyprocessors/json.go readJSON/readItems].

    ARGS_POST entries of a JSON request body, in the order readItems writes
    them into its result map: "json" + ".key" (object member, unescaped) or
    ".N" (array index) per level; strings unescaped, numbers / true / false
    as their raw text, null as ""; a non-empty array also writes its own
    key = element count after its elements.  Coraza then copies the Go map
    into ARGS_POST (case-sensitive keys, as MAP_VARS above) with
    SetIndex(key, 0, value) in (random) map order; this engine fixes the
    order to the first write of a key, holding the last value written.

    Read left to right; the first of these events decides:
      * a syntax error (not RFC 8259 JSON; gjson.Valid false) -> JsonBodyError;
      * an engine limit -> None (flagged unsupported): a scalar root value,
        nesting deeper than JSON_MAX_DEPTH, more than 4 x len(body) + 1024
        flattened bytes (every element's key, every string value that held
        escapes, every array count).
    The event order is the device parser's (kernels.hip parse_json_body)."""
    rd = _JsonReader(body)
    res: Dict[bytes, Tuple[bytes, bytes]] = {}
    lim = JSON_FLAT_LIMIT(len(body))
    flat = 0
    n = len(body)

    class _Limit(Exception):
        pass

    def put(key: bytes, val: bytes):
        res[key] = (key, val)

    try:
        rd.ws()
        if rd.i >= n:
            raise _JsonInvalid()
        c0 = body[rd.i]
        if c0 not in (0x7B, 0x5B):
            if c0 in b'"-0123456789tfn':
                return None  # a (possibly valid) scalar root: engine limit
            raise _JsonInvalid()
        # frame: [key, count, is_arr]
        st = [[b"json", 0, c0 == 0x5B]]
        rd.i += 1
        while st:
            F = st[-1]
            rd.ws()
            c = rd.peek()
            if c == (0x5D if F[2] else 0x7D):
                rd.i += 1
                if F[2] and F[1]:
                    cnt = str(F[1]).encode()
                    flat += len(cnt)
                    if flat > lim:
                        raise _Limit()
                    put(F[0], cnt)
                st.pop()
                continue
            if F[1]:
                rd.expect(0x2C)
                rd.ws()
            if F[2]:
                key = F[0] + b"." + str(F[1]).encode()
                flat += len(key)
                if flat > lim:
                    raise _Limit()
            else:
                name = rd.string()
                key = F[0] + b"." + name
                flat += len(key)
                if flat > lim:
                    raise _Limit()
                rd.ws()
                rd.expect(0x3A)
                rd.ws()
            F[1] += 1
            c = rd.peek()
            if c == 0x7B or c == 0x5B:
                if len(st) >= JSON_MAX_DEPTH:
                    raise _Limit()
                st.append([key, 0, c == 0x5B])
                rd.i += 1
            elif c == 0x22:
                v = rd.string()
                if rd.escaped:
                    flat += len(v)
                    if flat > lim:
                        raise _Limit()
                put(key, v)
            elif c in (0x74, 0x66, 0x6E):
                lit = b"true" if c == 0x74 else b"false" if c == 0x66 else b"null"
                if not rd.s.startswith(lit, rd.i):
                    raise _JsonInvalid()
                rd.i += len(lit)
                put(key, b"" if lit == b"null" else lit)
            else:
                put(key, rd.number())
        rd.ws()
        if rd.i != n:
            raise _JsonInvalid()
    except _JsonInvalid:
        raise JsonBodyError("invalid JSON")
    except _Limit:
        return None
    return list(res.values())


def go_atoi(s: bytes):
    """strconv.Atoi -> (value, ok)."""
    m = re.fullmatch(rb"[+-]?[0-9]+", s)
    if not m:
        return 0, False
    v = int(s)
    if v > 2**63 - 1 or v < -2**63:
        return (2**63 - 1 if v > 0 else -2**63), False
    return v, True


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


@dataclass
class Verdict:
    rule_id: int = 0
    status: int = 0
    action: str = ""
    phase: int = 0
    matched: List[int] = field(default_factory=list)
    tx: Dict[str, bytes] = field(default_factory=dict)
    unsupported: bool = False
    # every capture write in evaluation order: (top-level rule id, group, value)
    captures: List[Tuple[int, int, bytes]] = field(default_factory=list)


class Transaction:
    def __init__(self, cfg: WafConfig):
        self.cfg = cfg
        self.rule_engine = cfg.rule_engine
        self.body_access = cfg.request_body_access
        self.interruption: Optional[Tuple[int, int, str, int]] = None
        self.matched: List[int] = []
        self.tx: Dict[bytes, bytes] = {}       # lowercase key -> value
        self.skip_after = ""
        self.skip = 0
        self.allow = ""  # allow action in effect: "allow" | "allow:phase" | "allow:request"
        self.removed: List[Tuple[int, int]] = []
        self.removed_targets: List[Tuple[int, int, str, str]] = []
        self.single: Dict[str, bytes] = {k: b"" for k in SINGLE_VARS}
        self.single["REQBODY_ERROR"] = b"0"
        self.single["MULTIPART_STRICT_ERROR"] = b"0"
        self.maps: Dict[str, List[Tuple[bytes, bytes]]] = {
            "ARGS_GET": [], "ARGS_POST": [], "REQUEST_HEADERS": [],
            "REQUEST_COOKIES": [], "MATCHED_VARS": [], "XML": [], "FILES": [], "FILES_NAMES": [],
            "FILES_SIZES": [], "FILES_TMPNAMES": [], "MULTIPART_PART_HEADERS": []}
        self.force_body = False
        self.body = b""
        self.phase = 0
        self.cur_top = 0
        self.captures: List[Tuple[int, int, bytes]] = []
        self._tcache: Dict[Tuple[tuple, bytes], bytes] = {}

    # -- request population -------------------------------------------------
    def process_request(self, req: Request):
        v, args = process_uri(req.uri)
        self.single.update(v)
        self.single["REQUEST_METHOD"] = req.method
        self.single["REQUEST_PROTOCOL"] = req.proto
        self.single["REQUEST_LINE"] = req.method + b" " + req.uri + b" " + req.proto
        self.single["REMOTE_ADDR"] = req.remote_addr
        self.single["REMOTE_PORT"] = str(req.remote_port).encode()
        self.single["SERVER_NAME"] = req.server_name
        if len(args) > self.cfg.args_limit:
            # SecArgumentsLimit [upstream transaction.go AddGetRequestArgument]:
            # which arguments are dropped depends on Go's map order -- flagged
            raise UnsupportedInput("more ARGS_GET than SecArgumentsLimit")
        self.maps["ARGS_GET"] = list(args)
        for k, val in req.headers:
            if k == b"":
                continue
            self.maps["REQUEST_HEADERS"].append((k, val))
            kl = k.lower()
            if kl == b"content-type":
                vl = val.lower()
                if vl.startswith(b"application/x-www-form-urlencoded"):
                    self.single["REQBODY_PROCESSOR"] = b"URLENCODED"
                elif vl.startswith(b"multipart/form-data"):
                    self.single["REQBODY_PROCESSOR"] = b"MULTIPART"
            elif kl == b"cookie":
                self.maps["REQUEST_COOKIES"] += parse_cookies(val)
        self.body = req.body

    # -- collections ----------------------------------------------------------
    def _tx_items(self):
        return [(k, v) for k, v in self.tx.items()]

    def _collection(self, src):
        if src == "TX":
            return self._tx_items()
        return self.maps[src]

    def args_combined_size(self) -> bytes:
        """[upstream internal/collections/sized.go SizeCollection over ARGS_GET
        and ARGS_POST]: the sum of len(key) + len(value) of every entry."""
        return str(sum(len(k) + len(v) for src in ("ARGS_GET", "ARGS_POST") for k, v in self.maps[src])).encode()

    def get_field(self, rv: RuleVariable):
        """tx.GetField: returns list of (key, value)."""
        name = rv.name
        if name == "ARGS_COMBINED_SIZE":
            vals = [(b"", self.args_combined_size())]
        elif name in SINGLE_VARS:
            vals = [(b"", self.single.get(name, b""))]
        else:
            if name in MAP_VARS:
                srcs, ci = MAP_VARS[name]
                names = False
            else:
                srcs, ci = NAMES_VARS[name]
                names = True
            items = []
            for s in srcs:
                items += self._collection(s)
            if rv.key_rx is not None:
                items = [(k, v) for k, v in items
                         if rv.key_rx.match_string(k.lower() if ci else k)]
            elif rv.key:
                kk = rv.key.encode()
                if ci:
                    items = [(k, v) for k, v in items if k.lower() == kk.lower()]
                else:
                    items = [(k, v) for k, v in items if k == kk]
            if names:
                items = [(k, k) for k, v in items]
            vals = items
        if rv.exceptions:
            kept = []
            for k, v in vals:
                lk = k.lower()
                drop = False
                for ek, erx in rv.exceptions:
                    if erx is not None:
                        if erx.match_string(lk):
                            drop = True
                            break
                    elif ek.encode() == lk:
                        drop = True
                        break
                if not drop:
                    kept.append((k, v))
            vals = kept
        if rv.count:
            vals = [(b"", str(len(vals)).encode())]
        return vals

    # -- macros ---------------------------------------------------------------
    def expand(self, parts) -> bytes:
        out = b""
        for p in parts:
            if isinstance(p, str):
                out += p.encode()
                continue
            _, name, key = p
            if name == "TX":
                out += self.tx.get(key.encode(), b"")
            elif name == "ARGS_COMBINED_SIZE":
                out += self.args_combined_size()
            elif name in SINGLE_VARS:
                out += self.single.get(name, b"")
            elif name in MAP_VARS:
                srcs, ci = MAP_VARS[name]
                for s in srcs:
                    hit = [v for k, v in self._collection(s)
                           if (k.lower() == key.encode() if ci else k == key.encode())]
                    if hit:
                        out += hit[0]
                        break
            else:
                pass
        return out

    # -- operators ------------------------------------------------------------
    def eval_op(self, rule: Rule, value: bytes) -> bool:
        op = rule.op
        n = op.name
        if n == "rx":
            if rule.capture:
                m = op.rx.find_string_submatch(value)
                if m is None:
                    res = False
                else:
                    for i, c in enumerate(m):
                        if i == 9:
                            break
                        self.tx[str(i).encode()] = c
                        self.captures.append((self.cur_top, i, c))
                    res = True
            else:
                res = op.rx.match_string(value)
        elif n in ("pm", "pmfromfile"):
            low = value.lower()
            if rule.capture:
                caps = _pm_find_all(op.phrases, low, value)
                for i, c in enumerate(caps[:10]):
                    self.tx[str(i).encode()] = c
                    self.captures.append((self.cur_top, i, c))
                res = len(caps) > 0
            else:
                res = _pm_any(op, low)
        elif n == "contains":
            res = self.expand(op.macro) in value
        elif n == "containsword":
            w = self.expand(op.macro)
            res = _contains_word(value, w)
        elif n == "streq":
            res = value == self.expand(op.macro)
        elif n == "beginswith":
            res = value.startswith(self.expand(op.macro))
        elif n == "endswith":
            res = value.endswith(self.expand(op.macro))
        elif n == "within":
            res = value in self.expand(op.macro)
        elif n in ("eq", "ge", "gt", "le", "lt"):
            a, ok = go_atoi(self.expand(op.macro))
            if not ok:
                a = 0
            b, ok = go_atoi(value)
            if not ok:
                b = 0
            res = {"eq": b == a, "ge": b >= a, "gt": b > a, "le": b <= a, "lt": b < a}[n]
        elif n == "unconditionalmatch":
            res = True
        elif n == "nomatch":
            res = False
        elif n == "validatebyterange":
            res = any(not op.byte_ok[c] for c in value)
        elif n == "validateurlencoding":
            res = _invalid_url_encoding(value)
        elif n == "ipmatch":
            res = ipmatch(op.nets, value)
        elif n == "detectsqli":
            # detect_sqli.go: libinjection.IsSQLi; the fingerprint is captured as TX.0
            res, fp = libinjection.is_sqli(value)
            if res and rule.capture:
                self.tx[b"0"] = fp.encode()
                self.captures.append((self.cur_top, 0, fp.encode()))
        elif n == "detectxss":
            res = libinjection.is_xss(value)  # detect_xss.go
        elif n == "validateutf8encoding":
            try:
                value.decode("utf-8")
                res = False
            except UnicodeDecodeError:
                res = True
        else:
            raise AssertionError(n)
        return (not res) if op.negate else res

    # -- actions --------------------------------------------------------------
    def run_setvar(self, sv: SetVar):
        key = self.expand(sv.key).lower()
        if sv.remove:
            self.tx.pop(key, None)
            return
        value = self.expand(sv.value)
        cur = self.tx.get(key, b"")
        if len(value) == 0:
            self.tx[key] = b""
        elif value[:1] == b"+" or value[:1] == b"-":
            me, ok = go_atoi(cur)
            if not ok:
                me = 0
            vv, ok = go_atoi(value[1:])
            if not ok:
                return
            r = me + vv if value[:1] == b"+" else me - vv
            self.tx[key] = str(_wrap64(r)).encode()
        else:
            self.tx[key] = value

    def run_ctl(self, name: str, val: str):
        if name == "ruleremovebyid":
            for part in val.split(" "):
                part = part.strip()
                if not part:
                    continue
                if "-" in part:
                    a, b = part.split("-", 1)
                    self.removed.append((int(a), int(b)))
                else:
                    self.removed.append((int(part), int(part)))
        elif name in ("ruleremovebytag", "ruleremovebymsg"):
            # [upstream ctl.go]: tx.RemoveRuleByID for every rule whose tags
            # contain the value (whose msg equals it)
            for r in self.cfg.rules:
                if r.id and (val in r.tags if name == "ruleremovebytag" else r.msg == val):
                    self.removed.append((r.id, r.id))
        elif name in ("ruleremovetargetbytag", "ruleremovetargetbymsg"):
            sel, _, tgt = val.partition(";")
            sel = sel.strip()
            var, _, key = tgt.strip().partition(":")
            for r in self.cfg.rules:
                if r.id and (sel in r.tags if name == "ruleremovetargetbytag" else r.msg == sel):
                    self.removed_targets.append((r.id, r.id, var.strip().upper(), key.lower()))
        elif name == "ruleremovetargetbyid":
            # [upstream internal/actions/ctl.go]: "ID[-ID];VARIABLE[:key]" ->
            # tx.RemoveRuleTargetByID: rule.go doEvaluate adds (key) to the
            # variable's exceptions for rules with that id
            ids, _, tgt = val.partition(";")
            ids = ids.strip()
            if "-" in ids[1:]:
                a, b = ids.split("-", 1)
                lo, hi = int(a), int(b)
            else:
                lo = hi = int(ids)
            var, _, key = tgt.strip().partition(":")
            self.removed_targets.append((lo, hi, var.strip().upper(), key.lower()))
        elif name == "ruleengine":
            self.rule_engine = {"on": "On", "off": "Off", "detectiononly": "DetectionOnly"}[val.lower()]
        elif name == "requestbodyprocessor":
            self.single["REQBODY_PROCESSOR"] = val.upper().encode()
        elif name == "requestbodyaccess":
            self.body_access = val.lower() == "on"
        elif name == "forcerequestbodyvariable":
            self.force_body = val.lower() in ("on", "true", "1")

    def run_nondisruptive(self, rule: Rule):
        for kind, obj in rule.nondisruptive_order:
            if kind == "setvar":
                self.run_setvar(obj)
            elif kind == "ctl":
                self.run_ctl(*obj)

    def transform(self, rule: Rule, value: bytes) -> bytes:
        # transformations are pure: cached per (chain, value) for the transaction
        key = (tuple(rule.transforms), value)
        hit = self._tcache.get(key)
        if hit is not None:
            return hit
        v = value
        for t in rule.transforms:
            v = TRANSFORM_FNS[t](v)
        if len(self._tcache) < 65536:
            self._tcache[key] = v
        return v

    def match_variable(self, var: str, key: bytes, value: bytes):
        """[upstream transaction.go matchVariable]: MATCHED_VAR(_NAME) = the
        value and "VAR[:key]"; MATCHED_VARS(_NAMES) SetIndex(name, 0, value) --
        a name already there (case-insensitive keys) keeps its position."""
        name = var.encode() + (b":" + key if key else b"")
        self.single["MATCHED_VAR"] = value
        self.single["MATCHED_VAR_NAME"] = name
        mv = self.maps["MATCHED_VARS"]
        for j, (k, _) in enumerate(mv):
            if k.lower() == name.lower():
                mv[j] = (name, value)
                break
        else:
            mv.append((name, value))

    def do_evaluate(self, rule: Rule) -> int:
        """Rule.doEvaluate -> number of matched values (0 = no match)."""
        nmatch = 0
        if rule.op is None:
            nmatch = 1
            self.run_nondisruptive(rule)
        else:
            for rv in rule.variables:
                dyn = [key for lo, hi, var, key in self.removed_targets
                       if rule.id and lo <= rule.id <= hi and var == rv.name]
                if dyn:
                    rv = RuleVariable(rv.name, rv.key, rv.key_rx, rv.count,
                                      rv.exceptions + [(key, None) for key in dyn])
                for k, v in self.get_field(rv):
                    if rule.multimatch:
                        # rule.go executeTransformationsMultimatch: the value,
                        # then the value after each transformation that
                        # changed it (an unchanged step adds no candidate)
                        cands = [v]
                        for t in rule.transforms:
                            nv = TRANSFORM_FNS[t](v)
                            if nv != v:
                                cands.append(nv)
                                v = nv
                    else:
                        cands = [self.transform(rule, v)]
                    for tv in cands:
                        if self.eval_op(rule, tv):
                            nmatch += 1
                            self.match_variable(rv.name, k, tv)
                            self.run_nondisruptive(rule)
        if nmatch == 0:
            return 0
        if rule.parent_id == 0:
            nr = rule.chain
            while nr is not None:
                if self.do_evaluate(nr) == 0:
                    return 0
                nr = nr.chain
            # flow + disruptive actions (disruptive only with engine On)
            if rule.skip_after:
                self.skip_after = rule.skip_after
            if rule.skip:
                self.skip = rule.skip
            if rule.disruptive in ("deny", "drop", "redirect") and self.rule_engine == "On":
                self.interruption = (rule.id, rule.status, rule.disruptive, self.phase)
            elif rule.disruptive.startswith("allow") and self.rule_engine == "On":
                self.allow = rule.disruptive  # [upstream allow.go: tx.AllowType]
            if rule.id != 0:
                self.matched.append(rule.id)
        return nmatch

    def eval_phase(self, phase: int):
        """RuleGroup.Eval."""
        if self.rule_engine == "Off":
            return
        # [upstream] an earlier "allow" (every phase) or "allow:request" ends
        # the remaining request phases
        if self.allow in ("allow", "allow:request"):
            return
        self.phase = phase
        for r in self.cfg.rules:
            if self.interruption is not None:
                break
            if r.phase != 0 and r.phase != phase:
                continue
            if r.id != 0 and any(a <= r.id <= b for a, b in self.removed):
                continue
            if self.skip_after:
                if r.secmark == self.skip_after:
                    self.skip_after = ""
                continue
            if self.skip > 0:
                self.skip -= 1
                continue
            if r.secmark:
                continue
            # rulegroup.go: MATCHED_VARS(_NAMES) reset before each rule;
            # MATCHED_VAR(_NAME) keep the last match of the transaction
            self.maps["MATCHED_VARS"] = []
            self.cur_top = r.id
            self.do_evaluate(r)
            if self.allow:  # the allow rule ends this phase ("allow:phase": only this one)
                if self.allow == "allow:phase":
                    self.allow = ""
                break

    def process_request_body(self):
        if self.rule_engine == "Off":
            return
        if self.interruption is not None:
            return
        if self.body_access and len(self.body) > 0:
            # [upstream transaction.go WriteRequestBody]: a body over
            # SecRequestBodyLimit sets INBOUND_DATA_ERROR; with Reject the
            # transaction is interrupted with status 413 (no rule id) and
            # ProcessRequestBody never runs; with ProcessPartial only the first
            # SecRequestBodyLimit bytes are buffered.  ProcessRequestBody: a
            # buffer of exactly the limit sets INBOUND_DATA_ERROR too, and with
            # Reject returns before phase 2.  (DetectionOnly: no interruption,
            # nothing buffered; parity unpinned.)
            limit = self.cfg.request_body_limit
            reject = self.cfg.request_body_limit_action.lower() != "processpartial"
            if len(self.body) > limit:
                self.single["INBOUND_DATA_ERROR"] = b"1"
                if reject:
                    if self.rule_engine == "On":
                        self.interruption = (0, 413, "deny", 2)
                        return
                    self.body = b""
                else:
                    self.body = self.body[:limit]
            if len(self.body) >= limit and len(self.body) > 0:
                self.single["INBOUND_DATA_ERROR"] = b"1"
                if reject:
                    return
        if self.body_access and len(self.body) > 0:
            self.single["REQUEST_BODY_LENGTH"] = str(len(self.body)).encode()
            rbp = self.single.get("REQBODY_PROCESSOR", b"")
            if self.force_body:
                # [upstream transaction.go ProcessRequestBody]: forced variable
                # with no processor -> URLENCODED
                if rbp == b"":
                    rbp = b"URLENCODED"
                self.single["REQBODY_PROCESSOR"] = rbp
            if rbp == b"URLENCODED":
                self.single["REQUEST_BODY"] = self.body
                self.maps["ARGS_POST"] = parse_query(self.body)
            elif rbp == b"JSON":
                # [upstream json.go ProcessRequest]: ARGS_POST from readJSON,
                # the raw body kept as REQUEST_BODY.  A body that is not JSON:
                # readJSON's error -> generateRequestBodyError (REQBODY_ERROR
                # "1", REQBODY_ERROR_MSG "<processor>: <error>"), no ARGS_POST,
                # no REQUEST_BODY, and phase 2 still runs (CRS base rule
                # 200002 then denies with 400).
                try:
                    args = json_flatten(self.body)
                except JsonBodyError as e:
                    self.single["REQBODY_ERROR"] = b"1"
                    self.single["REQBODY_ERROR_MSG"] = b"JSON: " + str(e).encode()
                    args = []
                else:
                    if args is None:
                        raise UnsupportedInput("JSON body beyond the engine's limits")
                    self.single["REQUEST_BODY"] = self.body
                self.maps["ARGS_POST"] = args
            elif rbp == b"MULTIPART":
                # [upstream multipart.go ProcessRequest] (oracle/multipart.py);
                # an error -> MULTIPART_STRICT_ERROR and generateRequestBodyError,
                # the collections keep the parts before it; no REQUEST_BODY
                ct = b""
                for k, val in self.maps["REQUEST_HEADERS"]:
                    if k.lower() == b"content-type":
                        ct = val
                        break
                try:
                    res = multipart.process(self.body, ct)
                except multipart.MultipartUnsupported as e:
                    raise UnsupportedInput("multipart: %s" % e)
                self.maps["ARGS_POST"] = res["args_post"]
                self.maps["FILES"] = res["files"]
                self.maps["FILES_NAMES"] = res["files_names"]
                self.maps["FILES_SIZES"] = res["files_sizes"]
                self.maps["MULTIPART_PART_HEADERS"] = res["part_headers"]
                if res["combined_size"] is not None:
                    self.single["FILES_COMBINED_SIZE"] = res["combined_size"]
                if res["error"] is not None:
                    self.single["MULTIPART_STRICT_ERROR"] = b"1"
                    self.single["REQBODY_ERROR"] = b"1"
                    self.single["REQBODY_ERROR_MSG"] = b"MULTIPART: " + res["error"].encode()
            elif rbp == b"XML":
                # [upstream xml.go ProcessRequest] (oracle/xmlbody.py): XML
                # "//@*" = attribute values, "/*" = trimmed character data;
                # an error -> generateRequestBodyError, no XML values
                try:
                    attrs, content = xmlbody.read_xml(self.body)
                except xmlbody.XmlUnsupported as e:
                    raise UnsupportedInput("xml: %s" % e)
                except xmlbody.XmlError as e:
                    self.single["REQBODY_ERROR"] = b"1"
                    self.single["REQBODY_ERROR_MSG"] = b"XML: " + str(e).encode("latin-1")
                    attrs, content = [], []
                self.maps["XML"] = [(b"//@*", v) for v in attrs] + [(b"/*", v) for v in content]
            elif rbp == b"":
                pass
            else:
                raise UnsupportedInput("body processor %s" % rbp.decode())
        self.eval_phase(2)


def _pm_index(phrases):
    """(phrase set, distinct lengths longest first) of a phrase list."""
    key = id(phrases)
    ix = _PM_INDEX.get(key)
    if ix is None or ix[0] is not phrases:
        ps = set(phrases)
        ix = (phrases, ps, sorted({len(p) for p in ps}, reverse=True))
        _PM_INDEX[key] = ix
    return ix[1], ix[2]


_PM_INDEX = {}


def _pm_any(op, low: bytes) -> bool:
    """Some phrase occurs in low (the phrases are lowercased already)."""
    if len(op.phrases) <= 64:
        return any(p in low for p in op.phrases)
    ps, lens = _pm_index(op.phrases)
    if b"" in ps:
        return True
    for i in range(len(low)):
        for n in lens:
            if i + n <= len(low) and low[i:i + n] in ps:
                return True
    return False


def _pm_find_all(phrases, low: bytes, orig: bytes):
    """Leftmost-longest non-overlapping matches (aho-corasick MatchKind)."""
    ps, lens = _pm_index(phrases)
    out = []
    i = 0
    n = len(low)
    while i < n:
        best = 0
        for L in lens:  # longest first
            if L and i + L <= n and low[i:i + L] in ps:
                best = L
                break
        if best:
            out.append(orig[i:i + best])
            i += best
        else:
            i += 1
    return out


def _go_parse_ip(v: bytes):
    """Go net.ParseIP + IP.To4 via Python's ipaddress (an independent parser):
    (4, bytes) for IPv4 or an IPv4-mapped IPv6 address, (16, bytes), or None.
    Zones are rejected (ParseIP); IPv4 fields with leading zeros are rejected
    by both (netip)."""
    import ipaddress
    try:
        s = v.decode("ascii")
    except UnicodeDecodeError:
        return None
    if "%" in s or s.strip() != s or not s:
        return None
    try:
        a = ipaddress.ip_address(s)
    except ValueError:
        return None
    if a.version == 6 and a.ipv4_mapped is not None:
        return 4, a.ipv4_mapped.packed
    return (4 if a.version == 4 else 16), a.packed


def ipmatch_networks(arg: str):
    """[upstream coraza internal/operators/ipmatch.go]: comma-separated
    networks, a bare address gets /32 or /128, net.ParseCIDR (host bits
    masked off), invalid entries skipped.  IPNet.Contains compares To4() of
    the network number: a masked IPv4-mapped network is IPv4 with prefix-96."""
    import ipaddress
    nets = []
    for e in arg.split(","):
        e = e.strip()
        if not e:
            continue
        addr, _, bits = e.partition("/")
        got = _go_parse_ip(addr.encode())
        if got is None:
            continue
        fam = 4 if (":" not in addr) else 16
        if bits:
            if not bits.isdigit():
                continue
            nb = int(bits)
        else:
            nb = 32 if fam == 4 else 128
        if nb > 8 * fam:
            continue
        raw = ipaddress.ip_address(addr).packed
        netw = ipaddress.ip_network((raw, nb), strict=False)
        packed = netw.network_address.packed
        if fam == 16 and packed[:10] == b"\0" * 10 and packed[10:12] == b"\xff\xff":
            nets.append((4, packed[12:], max(0, nb - 96)))
        else:
            nets.append((fam, packed, nb))
    return nets


def ipmatch(nets, value: bytes) -> bool:
    got = _go_parse_ip(value)
    if got is None:
        return False
    fam, ip = got
    iv = int.from_bytes(ip, "big")
    for f, net, nb in nets:
        if f != fam:
            continue
        sh = 8 * f - nb
        if (iv >> sh) == (int.from_bytes(net, "big") >> sh):
            return True
    return False


def _contains_word(value: bytes, w: bytes) -> bool:
    if not w:
        return True
    i = value.find(w)
    while i >= 0:
        before = i == 0 or not (_isalnum(value[i - 1]) or value[i - 1] == 0x5F)
        j = i + len(w)
        after = j >= len(value) or not (_isalnum(value[j]) or value[j] == 0x5F)
        if before and after:
            return True
        i = value.find(w, i + 1)
    return False


def _invalid_url_encoding(d: bytes) -> bool:
    i, n = 0, len(d)
    while i < n:
        if d[i] == 0x25:
            if i + 2 >= n:
                return True
            if _ishex(d[i + 1]) and _ishex(d[i + 2]):
                i += 3
            else:
                return True
        else:
            i += 1
    return False


DEFAULT_TX_EXPORTS = (
    "blocking_inbound_anomaly_score", "inbound_anomaly_score_pl1",
    "inbound_anomaly_score_pl2", "inbound_anomaly_score_pl3",
    "inbound_anomaly_score_pl4", "detection_inbound_anomaly_score",
    "anomaly_score",
)


def inspect(cfg: WafConfig, req: Request, exports=DEFAULT_TX_EXPORTS) -> Verdict:
    """One full request: phase 1 then phase 2 (ProcessRequestHeaders/Body)."""
    tx = Transaction(cfg)
    out = Verdict()
    try:
        tx.process_request(req)
        tx.eval_phase(1)
        if tx.interruption is None:
            tx.process_request_body()
    except UnsupportedInput:
        out.unsupported = True
        return out
    if tx.interruption is not None:
        out.rule_id, out.status, out.action, out.phase = tx.interruption
    out.matched = list(tx.matched)
    out.captures = list(tx.captures)
    for name in exports:
        out.tx[name] = tx.tx.get(name.encode(), b"")
    return out


def compile_ruleset(configmaps: List[str]) -> WafConfig:
    """ruleset_controller.go:158-181: validate each ConfigMap, then join with
    '\\n' and compile the aggregate."""
    for text in configmaps:
        parse_seclang(text)
    return parse_seclang("\n".join(configmaps))
