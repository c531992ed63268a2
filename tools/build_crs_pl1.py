"""Build rulesets/crs_pl1.conf -- the C2/C3 benchmark ruleset.

Layout follows hack/generate_coreruleset_configmaps.py in the reference:
the BASE rules ConfigMap first (generate_coreruleset_configmaps.py:30-109,
transcribed below as data), then every rules/*.conf in sorted order
(:156), joined with "\\n" like the RuleSet controller does
(internal/controller/ruleset_controller.go:173-176).

The CRS v4.23.0 rule files themselves are downloaded by the reference's
Makefile (Makefile:185-206) and are not available offline, so rules/*.conf
here are the CRS-shaped files under rulesets/crs/ (see their headers).
"""
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# hack/generate_coreruleset_configmaps.py:36-109 (the `rules:` payload)
BASE_RULES = r'''SecRuleEngine On
SecRequestBodyAccess On
SecRequestBodyLimit 131072
SecRequestBodyInMemoryLimit 131072
SecRequestBodyLimitAction Reject
SecResponseBodyAccess Off
SecResponseBodyMimeType text/plain text/html text/xml
SecResponseBodyLimit 524288
SecResponseBodyLimitAction ProcessPartial
SecAuditEngine RelevantOnly
SecAuditLogType Serial
SecAuditLog /dev/stdout
SecAuditLogFormat JSON
SecAuditLogParts ABIJDEFHZ
SecAuditLogRelevantStatus "^(40[0-3]|40[5-9]|4[1-9][0-9]|5[0-9][0-9])$"
SecRule REQUEST_HEADERS:Content-Type "^(?:application(?:/soap\+|/)|text/)xml" \
 "id:200000,\
 phase:1,\
 t:none,t:lowercase,\
 pass,\
 nolog,\
 ctl:requestBodyProcessor=XML"
SecRule REQUEST_HEADERS:Content-Type "^application/json" \
 "id:200001,\
 phase:1,\
 t:none,t:lowercase,\
 pass,\
 nolog,\
 ctl:requestBodyProcessor=JSON"
SecRule REQUEST_HEADERS:Content-Type "^application/[a-z0-9.-]+[+]json" \
 "id:200006,\
 phase:1,\
 t:none,t:lowercase,\
 pass,\
 nolog,\
 ctl:requestBodyProcessor=JSON"
SecRule REQBODY_ERROR "!@eq 0" \
 "id:200002,\
 phase:2,\
 t:none,\
 log,\
 deny,\
 status:400,\
 msg:'Failed to parse request body.',\
 logdata:'%{reqbody_error_msg}',\
 severity:2"
SecRule MULTIPART_STRICT_ERROR "!@eq 0" \
 "id:200003,\
 phase:2,\
 t:none,\
 log,\
 deny,\
 status:400,\
 msg:'Multipart request body failed strict validation.'"
SecDefaultAction "phase:2,log,auditlog,deny,status:403"
SecAction \
 "id:900120,\
 phase:1,\
 pass,\
 t:none,\
 nolog,\
 tag:'OWASP_CRS',\
 ver:'OWASP_CRS/4.23.0',\
 setvar:tx.early_blocking=1"
SecAction \
 "id:900990,\
 phase:1,\
 pass,\
 t:none,\
 nolog,\
 tag:'OWASP_CRS',\
 ver:'OWASP_CRS/4.23.0',\
 setvar:tx.crs_setup_version=4230"
'''


def main():
    parts = [BASE_RULES]
    for p in sorted(glob.glob(os.path.join(ROOT, "rulesets", "crs", "*.conf"))):
        parts.append(open(p).read())
    out = os.path.join(ROOT, "rulesets", "crs_pl1.conf")
    with open(out, "w") as f:
        f.write("\n".join(parts))
    print("wrote", out, sum(len(p) for p in parts), "bytes")


if __name__ == "__main__":
    main()
