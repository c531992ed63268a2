// @detectSQLi / @detectXSS on the device: libinjection 3.x restated for one
// lane per value.
//
// [upstream] Coraza v3.3.3 internal/operators/detect_sqli.go / detect_xss.go
// call libinjection-go v0.2.2 (/root/reference/go.mod:24): IsSQLi tokenizes
// the value in up to five (quote, comment-dialect) contexts, folds the token
// stream to <= 5 tokens and looks the fingerprint up; IsXSS runs the HTML5
// tokenizer in five start states and tests tags / attributes / URLs against
// black lists.  The control flow below follows libinjection_sqli.c,
// libinjection_html5.c and libinjection_xss.c; the keyword table and the
// fingerprint grammar are authored (libinj_tables.py; PARITY UNPINNED).
//
// GPU shape: k_stream tests each (item, stream) value against an exact
// character-class prefilter (li_sqli_candidate / li_xss_candidate) and lists
// the candidates; k_detect runs these functions one lane per candidate with
// the tokenizer state in LDS; k_eval calls them when it re-evaluates a
// set-bit link exactly.  Tokens point into the value (or into the keyword
// pool after a word merge) instead of copying 32-byte values.
#pragma once
#include <stdint.h>

#include "libinj_words.h"

namespace gi {
#include "libinj_body.h"
}  // namespace gi
