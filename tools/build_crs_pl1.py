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


# hack/generate_coreruleset_configmaps.py:113-141: the X-CRS-Test rule block the
# generator appends to the base rules with --include-test-rule (:451-452), the
# go-ftw configuration (coraza-proxy-wasm ftw-config.conf): blocking paranoia
# level 4, DetectionOnly, and an X-CRS-Test header that disables detection
X_CRS_TEST_RULE = r'''SecResponseBodyMimeType text/plain text/html text/xml application/json
SecDefaultAction "phase:3,log,auditlog,pass"
SecDefaultAction "phase:4,log,auditlog,pass"
SecDefaultAction "phase:5,log,auditlog,pass"
SecDebugLogLevel 3
SecAction \
 "id:900005,\
 phase:1,\
 nolog,\
 pass,\
 t:none,\
 setvar:tx.blocking_paranoia_level=4,\
 setvar:tx.crs_validate_utf8_encoding=1,\
 setvar:tx.arg_name_length=100,\
 setvar:tx.arg_length=400,\
 setvar:tx.total_arg_length=64000,\
 setvar:tx.max_num_args=255,\
 setvar:tx.max_file_size=64100,\
 setvar:tx.combined_file_sizes=65535,\
 ctl:ruleEngine=DetectionOnly,\
 ctl:ruleRemoveById=910000"
SecRule REQUEST_HEADERS:X-CRS-Test "@rx ^.*$" \
 "id:999999,\
 pass,\
 phase:1,\
 log,\
 msg:'X-CRS-Test %{MATCHED_VAR}',\
 ctl:ruleRemoveById=1-999999"
'''

# C4: blocking paranoia level 4 (crs-setup.conf's 900000 convention)
PL4_SETUP = r'''SecAction \
 "id:900000,\
 phase:1,\
 pass,\
 t:none,\
 nolog,\
 tag:'OWASP_CRS',\
 ver:'OWASP_CRS/4.23.0',\
 setvar:tx.blocking_paranoia_level=4"
'''


def main():
    crs = [open(p).read() for p in sorted(glob.glob(os.path.join(ROOT, "rulesets", "crs", "*.conf")))]
    outs = {
        "crs_pl1.conf": [BASE_RULES] + crs,
        "crs_pl4.conf": [BASE_RULES + PL4_SETUP] + crs,
        "crs_ftw.conf": [BASE_RULES + "\n" + X_CRS_TEST_RULE] + crs,
    }
    for name, parts in outs.items():
        out = os.path.join(ROOT, "rulesets", name)
        with open(out, "w") as f:
            f.write("\n".join(parts))
        print("wrote", out, sum(len(p) for p in parts), "bytes")


if __name__ == "__main__":
    main()
