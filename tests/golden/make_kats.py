"""Generate tests/golden/kats.json -- the reference's own known-answer tests.

The reference evaluates rules only in its end-to-end cluster tests; these are
the request -> HTTP-status assertions (plus the "logged by rule N" notes of
the samples README) transcribed as data, each with the file:line it comes
from.  Rule texts are the ConfigMap payloads those tests create.

Run in the build container (where /root/reference exists):
    python tests/golden/make_kats.py
The samples RuleSet is read from /root/reference/config/samples/ruleset.yaml
with yaml.safe_load; everything else is transcribed literally below.
"""

import json
import os
import sys

import yaml

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def simple_block_rule(rid, target):
    # test/framework/resources.go:122-127
    return ('SecRule ARGS|REQUEST_URI|REQUEST_HEADERS "@contains %s" '
            '"id:%d,phase:2,deny,status:403,msg:\'%s blocked\'"' % (target, rid, target))


# Headers the Go test client (net/http) sends: test/framework/traffic.go:124
GO_HEADERS = [["Host", "localhost"], ["User-Agent", "Go-http-client/1.1"],
              ["Accept-Encoding", "gzip"]]
# Headers curl sends in config/samples/README.md:36-60
CURL_HEADERS = [["Host", "localhost:8080"], ["User-Agent", "curl/8.5.0"], ["Accept", "*/*"]]


def req(uri, status, matched=None, not_matched=None, headers=GO_HEADERS, src=""):
    return {"method": "GET", "uri": uri, "proto": "HTTP/1.1", "headers": headers,
            "body": "", "expect_status": status, "expect_matched": matched or [],
            "expect_not_matched": not_matched or [], "source": src}


def main():
    scenarios = []

    # --- test/integration/coreruleset_test.go:57-127 -----------------------
    crs_base = ("\nSecRuleEngine On\nSecRequestBodyAccess On\nSecResponseBodyAccess Off\n"
                "SecAuditLog /dev/stdout\nSecAuditLogFormat JSON\nSecAuditEngine RelevantOnly\n")
    crs_sqli = ('\nSecRule ARGS "@rx (?i:(\\b(select|union|insert|update|delete|drop)\\b.*\\b(from|into|where|table)\\b))" \\\n'
                '  "id:942100,\\\n  phase:2,\\\n  deny,\\\n  status:403,\\\n  t:none,t:urlDecodeUni,\\\n'
                '  msg:\'SQL Injection Attack Detected\',\\\n  severity:\'CRITICAL\'"\n')
    crs_xss = ('\nSecRule ARGS "@rx (?i:<script[^>]*>)" \\\n'
               '  "id:941100,\\\n  phase:2,\\\n  deny,\\\n  status:403,\\\n  t:none,t:urlDecodeUni,t:htmlEntityDecode,\\\n'
               '  msg:\'XSS Attack Detected\',\\\n  severity:\'CRITICAL\'"\n')
    scenarios.append({
        "name": "coreruleset_compatible",
        "source": "test/integration/coreruleset_test.go:57-127",
        "configmaps": [crs_base, crs_sqli, crs_xss],
        "requests": [
            req("/?id=1+UNION+SELECT+username+FROM+users", 403, [942100], src="coreruleset_test.go:121"),
            req("/?p=<script>alert(1)</script>", 403, [941100], src="coreruleset_test.go:124"),
            req("/?q=hello+world", 200, [], [942100, 941100], src="coreruleset_test.go:127"),
        ]})

    # --- test/integration/reconcile_test.go:43-88 --------------------------
    scenarios.append({
        "name": "reconcile_initial",
        "source": "test/integration/reconcile_test.go:43-68",
        "configmaps": ["SecRuleEngine On", simple_block_rule(3001, "evilmonkey")],
        "requests": [req("/?test=evilmonkey", 403, [3001], src="reconcile_test.go:67"),
                     req("/?test=safe", 200, [], [3001], src="reconcile_test.go:68")]})
    scenarios.append({
        "name": "reconcile_add_sinister",
        "source": "test/integration/reconcile_test.go:72-78",
        "configmaps": ["SecRuleEngine On", simple_block_rule(3001, "evilmonkey"),
                       simple_block_rule(3002, "sinistermonkey")],
        "requests": [req("/sinistermonkey", 403, [3002], src="reconcile_test.go:78")]})
    scenarios.append({
        "name": "reconcile_replace_maniacal",
        "source": "test/integration/reconcile_test.go:82-88",
        "configmaps": ["SecRuleEngine On", simple_block_rule(3001, "evilmonkey"),
                       simple_block_rule(3002, "maniacalmonkey")],
        "requests": [req("/sinistermonkey", 200, [], [3002], src="reconcile_test.go:87"),
                     req("/maniacalmonkey", 403, [3002], src="reconcile_test.go:88")]})

    # --- test/integration/multiple_gateways_test.go:46-100 -----------------
    scenarios.append({
        "name": "multiple_gateways",
        "source": "test/integration/multiple_gateways_test.go:46-100",
        "configmaps": ["SecRuleEngine On", simple_block_rule(1001, "blocked")],
        "requests": [req("/?test=blocked", 403, [1001], src="multiple_gateways_test.go:89"),
                     req("/?test=safe", 200, [], [1001], src="multiple_gateways_test.go:100")]})

    # --- test/integration/multi_engine_gateway_test.go ---------------------
    scenarios.append({
        "name": "engine_per_gateway_shared_ruleset",
        "source": "test/integration/multi_engine_gateway_test.go:51-84",
        "configmaps": ["SecRuleEngine On", simple_block_rule(1001, "evil")],
        "requests": [req("/?test=evil", 403, [1001], src="multi_engine_gateway_test.go:82"),
                     req("/?test=safe", 200, [], [1001], src="multi_engine_gateway_test.go:83")]})
    # two engines on one gateway: each RuleSet is evaluated on its own; the
    # gateway blocks if either blocks (multi_engine_gateway_test.go:102-138)
    for which, rid, word in (("a", 2001, "attackA"), ("b", 2002, "attackB")):
        other = "attackB" if which == "a" else "attackA"
        scenarios.append({
            "name": "multiple_engines_single_gateway_ruleset_" + which,
            "source": "test/integration/multi_engine_gateway_test.go:102-138",
            "configmaps": ["SecRuleEngine On", simple_block_rule(rid, word)],
            "requests": [req("/?test=" + word, 403, [rid], src="multi_engine_gateway_test.go:136-137"),
                         req("/?test=" + other, 200, [], [rid], src="multi_engine_gateway_test.go:136-137"),
                         req("/?test=safe", 200, [], [rid], src="multi_engine_gateway_test.go:138")]})

    # --- config/samples/ruleset.yaml + config/samples/README.md:36-60 ------
    docs = list(yaml.safe_load_all(open(os.path.join(REF, "config/samples/ruleset.yaml"))))
    cms = {d["metadata"]["name"]: d["data"]["rules"] for d in docs if d["kind"] == "ConfigMap"}
    rs = [d for d in docs if d["kind"] == "RuleSet"][0]
    order = [r["name"] for r in rs["spec"]["rules"]]
    sample_cms = [cms[n] for n in order]
    scenarios.append({
        "name": "samples_ruleset",
        "source": "config/samples/ruleset.yaml:1-81, config/samples/README.md:36-60",
        "configmaps": sample_cms,
        "requests": [
            req("/", 200, [], [1001, 2001, 3001], headers=CURL_HEADERS, src="README.md:42"),
            req("/?q=evilmonkey", 403, [3001], headers=CURL_HEADERS, src="README.md:48"),
            req("/?q=select+*+from+users", 200, [1001], [3001], headers=CURL_HEADERS, src="README.md:51-54"),
            req("/?q=<script>alert(1)</script>", 200, [2001], [3001], headers=CURL_HEADERS, src="README.md:57-60"),
        ]})

    out = {"generator": "tests/golden/make_kats.py", "scenarios": scenarios}
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(out, f, indent=1)
    # the samples ruleset is also the C1 bench/parity workload
    with open(os.path.join(HERE, "samples_ruleset.conf"), "w") as f:
        f.write("\n".join(sample_cms))
    print("wrote", len(scenarios), "scenarios", file=sys.stderr)


if __name__ == "__main__":
    main()
