"""SecLang surface beyond the rule loop: what the reference's RuleSet text can
carry besides request-phase SecRules.

* The generator keeps every CRS *.conf (hack/generate_coreruleset_configmaps.py:156),
  including RESPONSE-950..980 (phases 3-5): NewWAF accepts them
  (ruleset_controller.go:159-160), the request path never evaluates them.
* A RuleSet aggregates arbitrary ConfigMaps (ruleset_controller.go:142-176), so
  operators' tuning directives land in the same text: SecRuleRemoveBy{Id,Tag,Msg},
  SecRuleUpdateTargetBy{Id,Tag,Msg}, SecRuleUpdateActionById, ctl:ruleRemove*By{Tag,Msg},
  allow, SERVER_NAME, SecArgumentsLimit.
* RuleGroup.Add rejects a repeated rule id.

CPU tests: both compilers accept / reject the same text with the same class of
error.  GPU tests (-m gpu): bit-exact verdicts against the oracle.
"""
import os

import pytest

import gpuinspect
import traffic
from oracle import compare, coraza

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRS = os.path.join(ROOT, "rulesets", "crs_pl1.conf")


def _both(text):
    """(engine error code or 0, oracle exception class name or "")."""
    try:
        gpuinspect.Ruleset(text)
        code = 0
    except gpuinspect.SecLangError as e:
        code = e.code
    try:
        coraza.parse_seclang(text)
        oerr = ""
    except coraza.SecLangError as e:
        oerr = type(e).__name__
    return code, oerr


def test_crs_ruleset_keeps_response_files():
    text = open(CRS).read()
    assert "RESPONSE_BODY" in text and "phase:4" in text and "id:959100" in text
    assert _both(text) == (0, "")
    # the request-path program holds no response-phase rule
    cfg = coraza.parse_seclang(text)
    ids = {r.id for r in cfg.rules if r.phase >= 3}
    assert 959100 in ids and 950130 in ids


def test_duplicate_rule_id_rejected():
    a = 'SecRule ARGS "@rx a" "id:10,phase:1,pass"\n'
    assert _both(a + 'SecRule ARGS "@rx b" "id:10,phase:2,pass"') == (gpuinspect.GI_EPARSE, "SecLangError")
    # chain links carry no id of their own; a removed id may be reused
    assert _both(a + 'SecRule ARGS "@rx b" "id:11,phase:1,pass,chain"\nSecRule ARGS "@rx c" "t:none"') == (0, "")
    assert _both(a + "SecRuleRemoveById 10\n" + 'SecRule ARGS "@rx b" "id:10,phase:2,pass"') == (0, "")


def test_crs_rule_ids_unique():
    for name in ("crs_pl1", "crs_pl4", "crs_ftw"):
        cfg = coraza.parse_seclang(open(os.path.join(ROOT, "rulesets", name + ".conf")).read())
        ids = [r.id for r in cfg.rules if r.id]
        assert len(ids) == len(set(ids)), name


@pytest.mark.parametrize("rule,want", [
    # a response variable / operator / transformation in a request-phase rule
    ('SecRule RESPONSE_BODY "@rx x" "id:1,phase:2,deny"', (gpuinspect.GI_EUNSUPPORTED, "SecLangUnsupported")),
    ('SecRule ARGS "@verifyCC \\d{16}" "id:1,phase:2,deny"', (gpuinspect.GI_EUNSUPPORTED, "SecLangUnsupported")),
    ('SecRule ARGS "@rx x" "id:1,phase:1,deny,t:uppercase"', (gpuinspect.GI_EUNSUPPORTED, "SecLangUnsupported")),
    # ... is fine in phases 3-5
    ('SecRule RESPONSE_BODY "@rx x" "id:1,phase:4,deny"', (0, "")),
    ('SecRule RESPONSE_HEADERS:Content-Type "@verifyCC \\d{16}" "id:1,phase:3,deny,t:uppercase"', (0, "")),
    ('SecRule RESPONSE_STATUS "!@rx ^404$" "id:1,phase:4,pass,chain"\nSecRule RESPONSE_BODY "@rx x" "t:none"', (0, "")),
    # syntax errors on both sides
    ('SecRule ARGS "@notAnOperator x" "id:1,phase:2,deny"', (gpuinspect.GI_EPARSE, "SecLangError")),
    ('SecRule ARGS "@rx x" "id:1,phase:2,allow:sometimes"', (gpuinspect.GI_EPARSE, "SecLangError")),
    ('SecRule ARGS "@rx x" "id:1,phase:2,ctl:noSuchCtl=1"', (gpuinspect.GI_EPARSE, "SecLangError")),
    ('SecRule ARGS "@rx x" "id:1,phase:2,t:noSuchTransform"', (gpuinspect.GI_EPARSE, "SecLangError")),
    ('SecRule NO_SUCH_VAR "@rx x" "id:1,phase:2,deny"', (gpuinspect.GI_EPARSE, "SecLangError")),
    ("SecRuleUpdateTargetById 42 \"!ARGS:x\"", (gpuinspect.GI_EPARSE, "SecLangError")),
    ("SecArgumentsLimit lots", (gpuinspect.GI_EPARSE, "SecLangError")),
    # log-only ctl options and actions are accepted
    ('SecRule ARGS "@rx x" "id:1,phase:2,pass,ctl:auditLogParts=+E,sanitiseRequestHeader:Authorization"', (0, "")),
])
def test_accept_reject_same_class(rule, want):
    assert _both(rule) == want


def test_remove_and_update_directives_oracle():
    text = "\n".join([
        'SecRule ARGS "@rx a" "id:1,phase:1,pass,tag:\'t-a\',msg:\'m one\'"',
        'SecRule ARGS "@rx b" "id:2,phase:1,pass,tag:\'t-b\'"',
        'SecRule ARGS "@rx c" "id:3,phase:2,pass,tag:\'t-a\'"',
        'SecRule ARGS "@rx d" "id:4,phase:2,deny,status:403"',
        'SecRule ARGS|REQUEST_HEADERS "@rx e" "id:5,phase:2,deny,status:403"',
        'SecRule ARGS "@rx f" "id:6,phase:2,pass"',
        "SecRuleRemoveByTag t-b",
        'SecRuleRemoveByMsg "m one"',
        "SecRuleUpdateActionById 4 \"pass,t:lowercase\"",
        "SecRuleUpdateTargetById 5 \"!ARGS:skip|REQUEST_COOKIES\"",
        'SecRuleUpdateTargetByTag "t-a" "!ARGS:q"',
        "SecRuleRemoveById 6-7",
    ])
    cfg = coraza.parse_seclang(text)
    assert [r.id for r in cfg.rules] == [3, 4, 5]
    r3, r4, r5 = cfg.rules
    assert r4.disruptive == "pass" and r4.transforms == ["lowercase"]
    assert [v.name for v in r5.variables] == ["ARGS", "REQUEST_HEADERS", "REQUEST_COOKIES"]
    assert r5.variables[0].exceptions == [("skip", None)]
    assert r3.variables[0].exceptions == [("q", None)]
    assert _both(text) == (0, "")


# ----------------------------------------------------------------- GPU parity
SURFACE_RULES = r'''SecRuleEngine On
SecRequestBodyAccess On
SecDefaultAction "phase:2,log,auditlog,deny,status:403"
SecArgumentsLimit 6
SecRule REQUEST_HEADERS:X-Allow "@streq all" "id:100,phase:1,allow,msg:'allow all'"
SecRule REQUEST_HEADERS:X-Allow "@streq phase" "id:101,phase:1,allow:phase"
SecRule REQUEST_HEADERS:X-Allow "@streq request" "id:102,phase:1,allow:request"
SecRule ARGS:late "@streq allow" "id:103,phase:2,allow"
SecRule REQUEST_HEADERS:X-Skip "@streq sqli" "id:110,phase:1,pass,nolog,ctl:ruleRemoveByTag=attack-sqli"
SecRule REQUEST_HEADERS:X-Skip "@streq msg" "id:111,phase:1,pass,nolog,ctl:ruleRemoveByMsg=XSS probe"
SecRule REQUEST_HEADERS:X-Skip "@streq tgt" "id:112,phase:1,pass,nolog,ctl:ruleRemoveTargetByTag=attack-sqli;ARGS:q"
SecRule REQUEST_HEADERS:X-Skip "@streq tgtmsg" "id:113,phase:1,pass,nolog,ctl:ruleRemoveTargetByMsg=XSS probe;ARGS:q"
SecRule SERVER_NAME "@streq admin.example.com" "id:120,phase:1,deny,status:401,msg:'admin host'"
SecRule SERVER_NAME "@rx ^internal\." "id:121,phase:2,pass,setvar:'tx.internal=1'"
SecRule ARGS "@rx (?i)union\s+select" "id:200,phase:2,block,tag:'attack-sqli',tag:'OWASP_CRS',msg:'SQLi probe'"
SecRule ARGS "@rx (?i)or\s+1=1" "id:201,phase:2,block,tag:'attack-sqli'"
SecRule ARGS "@rx (?i)<script" "id:202,phase:2,block,tag:'attack-xss',msg:'XSS probe'"
SecRule ARGS "@rx evilmonkey" "id:203,phase:2,deny,status:406,tag:'custom'"
SecRule REQUEST_HEADERS|ARGS "@rx sinister" "id:204,phase:2,deny,status:407"
SecRule ARGS "@rx benign" "id:205,phase:1,deny,status:408"
SecRule ARGS "@rx ^drop$" "id:206,phase:2,drop"
SecRuleUpdateTargetById 204 "!ARGS:note|!REQUEST_HEADERS:referer"
SecRuleUpdateActionById 205 "pass,setvar:'tx.benign=1'"
SecRuleUpdateTargetByTag custom "!ARGS:ok"
SecRule ARGS "@rx gone" "id:300,phase:2,deny,status:409,tag:'legacy'"
SecRuleRemoveByTag legacy
SecRule TX:internal "@eq 1" "id:400,phase:2,pass,setvar:'tx.anomaly_score=+5'"
SecRule TX:benign "@eq 1" "id:401,phase:2,pass,setvar:'tx.anomaly_score=+1'"
SecRule RESPONSE_BODY "@rx secret" "id:500,phase:4,deny,status:500"
'''


def _surface_requests():
    heads = [[], [("X-Allow", "all")], [("X-Allow", "phase")], [("X-Allow", "request")],
             [("X-Skip", "sqli")], [("X-Skip", "msg")], [("X-Skip", "tgt")], [("X-Skip", "tgtmsg")],
             [("Referer", "sinister")], [("X-Note", "sinister")]]
    queries = ["q=1+union+select+x", "q=<script>", "a=1+or+1=1&q=x", "ok=evilmonkey", "x=evilmonkey",
               "note=sinister", "z=sinister", "w=benign", "late=allow&q=<script>", "v=drop", "y=gone",
               "a=1&b=2&c=3&d=4&e=5&f=6", "a=1&b=2&c=3&d=4&e=5&f=6&g=7", "q=plain"]
    servers = ["", "admin.example.com", "internal.example.com", "www.example.com"]
    txs = []
    k = 0
    for h in heads:
        for q in queries:
            t = gpuinspect.Transaction(method=b"GET", uri=("/p?" + q).encode())
            t.add_request_header("Host", "h")
            for a, b in h:
                t.add_request_header(a, b)
            t.set_server_name(servers[k % len(servers)])
            k += 1
            txs.append(t)
    # the same over POST bodies (phase-2 rules read ARGS_POST)
    for q in queries:
        t = gpuinspect.Transaction(method=b"POST", uri=b"/form")
        t.add_request_header("Content-Type", "application/x-www-form-urlencoded")
        t.add_request_header("X-Allow", "phase" if "late" in q else "none")
        t.write_request_body(q.encode())
        txs.append(t)
    return txs


def test_surface_oracle_semantics():
    """The oracle's reading of the new constructs on a few hand-checked requests."""
    cfg = coraza.parse_seclang(SURFACE_RULES)

    def run(q, headers=(), server=b""):
        return coraza.inspect(cfg, coraza.Request(b"GET", b"/p?" + q, b"HTTP/1.1",
                                                  [(b"Host", b"h")] + list(headers), b"", b"", 0, server))
    v = run(b"q=1+union+select+x")
    assert (v.rule_id, v.status) == (200, 403)
    v = run(b"q=1+union+select+x", [(b"X-Allow", b"all")])
    assert v.rule_id == 0 and 100 in v.matched and 200 not in v.matched
    v = run(b"q=1+union+select+x", [(b"X-Allow", b"phase")])  # allow:phase: phase 2 still runs
    assert v.rule_id == 200 and 101 in v.matched
    v = run(b"q=1+union+select+x", [(b"X-Allow", b"request")])
    assert v.rule_id == 0
    v = run(b"q=1+union+select+x", [(b"X-Skip", b"sqli")])  # ctl:ruleRemoveByTag=attack-sqli
    assert v.rule_id == 0
    v = run(b"q=1+union+select+x", [(b"X-Skip", b"tgt")])  # ARGS:q removed from the sqli rules
    assert v.rule_id == 0
    v = run(b"q=<script>", [(b"X-Skip", b"msg")])
    assert v.rule_id == 0
    v = run(b"x=evilmonkey")
    assert (v.rule_id, v.status) == (203, 406)
    v = run(b"ok=evilmonkey")  # SecRuleUpdateTargetByTag custom "!ARGS:ok"
    assert v.rule_id == 0
    v = run(b"note=sinister")  # SecRuleUpdateTargetById 204 "!ARGS:note"
    assert v.rule_id == 0
    v = run(b"w=benign")  # SecRuleUpdateActionById 205 "pass,..."
    assert v.rule_id == 0 and v.matched == [205, 401]
    v = run(b"y=gone")  # SecRuleRemoveByTag legacy
    assert v.rule_id == 0
    v = run(b"q=plain", server=b"admin.example.com")
    assert (v.rule_id, v.phase) == (120, 1)
    v = run(b"a=1&b=2&c=3&d=4&e=5&f=6&g=7")  # more ARGS_GET than SecArgumentsLimit
    assert v.unsupported


@pytest.mark.gpu
def test_gpu_surface_parity():
    rs = gpuinspect.Ruleset(SURFACE_RULES)
    batch = gpuinspect.pack(_surface_requests())
    eng = gpuinspect.Engine(rs, matched_cap=64)
    res = eng.inspect(batch)
    cfg = coraza.parse_seclang(SURFACE_RULES)
    orc = compare.oracle_verdicts(cfg, batch, rs.exports)
    assert not compare.compare(res, orc)
    acts = {int(a) for a in res.verdicts["action"]}
    assert acts >= {0, 1, 2}
    n_uns = sum(1 for v in orc.values() if v.unsupported)
    assert 0 < n_uns < batch.n_req // 4  # only the over-limit requests


@pytest.mark.gpu
def test_gpu_crs_with_tuning_configmap():
    """CRS PL1 aggregated with an operator's tuning ConfigMap (exclusions by
    tag and target, an allow-listed path), as ruleset_controller.go:173-176
    joins them, over the mixed GET/POST traffic."""
    tuning = "\n".join([
        'SecRule REQUEST_URI "@beginsWith /api/" "id:1001,phase:1,pass,nolog,ctl:ruleRemoveByTag=attack-sqli"',
        'SecRule REQUEST_URI "@beginsWith /search" "id:1002,phase:1,pass,nolog,ctl:ruleRemoveTargetByTag=attack-xss;ARGS:q"',
        'SecRule REQUEST_HEADERS:User-Agent "@streq healthcheck" "id:1003,phase:1,allow,nolog"',
        'SecRuleUpdateTargetById 942100 "!ARGS:id"',
        "SecRuleRemoveById 920350",
    ])
    text = gpuinspect.aggregate_configmaps([open(CRS).read(), tuning])
    rs = gpuinspect.Ruleset(text)
    batch = traffic.TrafficGen(traffic.SEED + 55).batch(600, post_frac=0.3, attack_rate=0.4)
    eng = gpuinspect.Engine(rs, matched_cap=128)
    res = eng.inspect(batch)
    cfg = coraza.parse_seclang(text)
    orc = compare.oracle_verdicts(cfg, batch, rs.exports)
    bad = compare.compare(res, orc)
    assert not bad, bad
    assert int((res.verdicts["action"] != 0).sum()) > 20
