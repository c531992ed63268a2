// GPU artifact of a compiled RuleSet: the whole host Program (rule records,
// automata, LDS job images, scan plan) as one versioned, checksummed blob.
//
// The operator compiles a RuleSet once per cache UUID and serves the blob
// next to RuleSetEntry.Rules (internal/rulesets/cache/cache.go:32-36); a data
// plane that polls GET /rules/<key>/latest (server.go:163-181) loads it with
// gi_ruleset_load instead of recompiling the SecLang text.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "compile.h"

namespace gi {

constexpr uint32_t kArtifactVersion = 6;

// FNV-1a 64 (artifact checksum and SecLang source digest).
uint64_t fnv64(const uint8_t* p, size_t n, uint64_t h = 1469598103934665603ull);

std::vector<uint8_t> serialize_program(const Program& P);
// false + *err on a malformed, truncated, corrupted or foreign-version blob.
bool deserialize_program(const uint8_t* buf, size_t n, Program* P, std::string* err);
// Cross-reference check of a Program: every index and offset a kernel
// dereferences (rule / variable / operator / action / template records,
// automata tables, LDS job images, scan plan, hit slots, TX slots) lies inside
// its table.  false + *err names the first violation.
bool validate_program(const Program& P, std::string* err);

}  // namespace gi
