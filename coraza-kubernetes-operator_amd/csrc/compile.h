// Host-side compiled RuleSet (before upload).  See compile.cpp.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "gi_program.h"
#include "regex.h"

namespace gi {

// Compiler revision: bumped on every change to what a given SecLang text
// compiles to (record semantics, phase-A eligibility, capture policy, ...),
// even when the record layout stays the same.  gi_compile folds it into the
// source digest and the artifact stores it, so an artifact written by another
// compiler revision is rejected (and recompiled from the rules text).
constexpr const char* kCompilerRev = "gi-seclang-compiler/18";

struct Program {
  std::vector<DRule> rules;
  std::vector<uint32_t> top;
  std::vector<DVarRef> vars;
  std::vector<DExc> excs;
  std::vector<DOp> ops;
  std::vector<DAction> acts;
  std::vector<DTmplPart> tparts;
  std::vector<DTmpl> tmpls;
  std::vector<uint8_t> tchains;
  std::vector<DDfa> dfas;
  std::vector<DNfa> nfas;
  std::vector<uint16_t> trans;
  std::vector<uint8_t> u8pool;
  std::vector<uint32_t> nranges;
  std::vector<uint8_t> strpool;
  std::vector<uint32_t> slot_names;  // (off, len) pairs into strpool
  std::vector<uint64_t> u64pool;     // union-automaton accept masks
  std::vector<DStream> streams;      // phase-A scan plan
  std::vector<DFilter> filters;      // global (deduplicated) phase-A variable filters
  std::vector<uint8_t> sfilt;        // per stream filter: global filter id
  uint8_t item_sides[8] = {0};       // per FieldKind: bit0 value side, bit1 key side is filtered
  uint32_t item_singles = 0;         // single variables some filter reads (1 << SingleId)
  std::vector<uint32_t> body_links;    // phase>=2 phase-A links with a residual REQUEST_BODY target (k_body)
  std::vector<uint32_t> always_slots;  // hit slots without an automaton image (always set)
  std::vector<DJob> jobs;
  std::vector<DJobDfa> jdfas;
  std::vector<DPat> pats;
  std::vector<DScanVal> svals;
  std::vector<uint8_t> images;
  std::vector<DPike> pikes;            // submatch programs of observable captures
  std::vector<DPikeInst> pike_insts;
  std::vector<uint32_t> pike_ranges;
  std::vector<DDynSite> dyn_sites;     // macro-key setvars (run-time TX keys)
  std::vector<uint32_t> txrx;          // static slots each regex-keyed TX target matches
  std::vector<DSnapSlot> tx_snap;      // folded TX state after the request-independent phase-1 prefix
  std::vector<uint32_t> fold_ids;      // rule ids that prefix matched
  std::vector<uint32_t> rule_groups;   // per rule record: ctl removal-group mask (ByTag / ByMsg); [0] when none
  uint32_t n_rm_groups = 0;
  uint32_t args_limit = 1000;          // SecArgumentsLimit
  std::vector<uint32_t> fold_runs;     // per run of folded phase-1 rules: ids offset, id count, walk end,
                                       // skipAfter marker pending at the end (0xFFFFFFFF: none)
  uint32_t fold_nids = 0;              // fold_ids entries (the section holds a placeholder when 0)
  uint8_t fold_on = 0;
  uint32_t max_tx_lit = 0;             // longest literal a setvar can store (MATCHED_VARS arena bound)
  uint32_t n_hit_slots = 0;
  uint32_t n_union_dfas = 0;
  uint32_t max_img_bytes = 0;      // largest small-job LDS image
  uint32_t max_big_img_bytes = 0;  // largest big-job LDS image
  std::string plan_json;             // human-readable scan plan (gi_ruleset_describe)
  std::vector<int32_t> exports;
  std::vector<std::string> export_names;
  uint32_t n_slots = 0, n_markers = 0;
  uint8_t rule_engine = 1, body_access = 0;
  uint8_t mv_used = 0;  // some target / macro reads the matched-variable state
  uint8_t body_partial = 0;  // SecRequestBodyLimitAction ProcessPartial
  uint64_t body_limit = 134217728;
  uint64_t source_digest = 0;  // FNV-1a 64 of the SecLang text and the export list (artifact identity)
};

// Returns 0, -1 (parse error) or -2 (unsupported); *err holds the message.
// data_files: @pmFromFile contents by the name the rule gives (Coraza reads
// them from the rules' directory; here the caller supplies them).
int compile_program(const std::string& text, const std::vector<std::string>& exports, uint32_t dfa_cap,
                    Program* out, std::string* err,
                    const std::map<std::string, std::string>* data_files = nullptr);

}  // namespace gi
