// RE2-syntax (Go regexp/syntax, Perl flags) parser and automaton builders.
//
// Replaces, on the compile side, what coraza/v3 v3.3.3 does in
// internal/operators/rx.go (`regexp.Compile("(?sm)" + arg)`) and
// internal/operators/pm.go (aho-corasick, ASCII case-insensitive)
// [upstream, not vendored; see DESIGN.md].  Call site in the reference:
// internal/controller/ruleset_controller.go:159-160 (coraza.NewWAF compiles
// every @rx / @pm of a RuleSet).
//
// Output is a DFA over an alphabet of *rune classes*: Go matches over runes
// (invalid UTF-8 bytes decode as U+FFFD, one byte each), so the device scan
// decodes UTF-8 exactly like utf8.DecodeRune and maps each rune to its class
// (ASCII through a 128-entry table, non-ASCII through sorted ranges).  Phrase
// automata (@pm/@contains) run in byte mode instead.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace gi {

struct RuneRange {
  uint32_t lo, hi;
};
using RuneSet = std::vector<RuneRange>;  // sorted, non-overlapping, merged

enum NodeKind : uint8_t { N_CLASS, N_CAT, N_ALT, N_REPEAT, N_CAPTURE, N_EMPTY, N_ASSERT };

enum AssertKind : uint8_t {
  AS_BOT = 1,   // \A, ^ without (?m)
  AS_EOT = 2,   // \z, $ without (?m)
  AS_BOL = 4,   // ^ with (?m)
  AS_EOL = 8,   // $ with (?m)
  AS_WB = 16,   // \b (ASCII word chars)
  AS_NWB = 32,  // \B
};

struct ReNode {
  NodeKind kind;
  RuneSet set;            // N_CLASS
  std::vector<int> kids;  // N_CAT / N_ALT; N_REPEAT / N_CAPTURE use kids[0]
  int min = 0, max = 0;   // N_REPEAT (max == -1: unbounded)
  bool greedy = true;
  int cap = 0;
  uint8_t assert_kind = 0;
};

struct Regex {
  std::vector<ReNode> nodes;
  int root = -1;
  int ncap = 0;
};

// Parse `pattern` with Go regexp/syntax Perl flags.  Returns false + message
// on syntax Go would reject, or on constructs this engine does not support
// (\p{..} Unicode groups).
bool re_parse(const std::string& pattern, Regex* out, std::string* err);

// Two automaton shapes share this struct:
//  * single (multi == false): sticky-accept DFA; once `accept` is entered the
//    scan can stop (match).  end_accept[s]: match at end of input.
//  * multi  (multi == true): union of n_pat patterns, no sticky state.  A
//    transition whose u16 has bit 15 set completes matches *before* consuming
//    the class; the matched set is acc[5*s + cls_combo[cls]] (combo = bit0
//    next-is-'\n', bit1 next-is-word, the only facts ^ $ \b \B look at).
//    acc[5*s + 4] is the set matched at end of input.
struct Dfa {
  uint32_t n_states = 0, n_classes = 0, start = 0, accept = 0;
  bool byte_mode = false;               // phrase automata: bytes, no UTF-8 decode
  bool multi = false;
  uint32_t n_pat = 1;
  std::vector<uint16_t> trans;          // n_states * n_classes
  std::vector<uint8_t> end_accept;      // per state: matches at end of input (single)
  std::vector<uint8_t> amap;            // 128 (rune mode) or 256 (byte mode)
  std::vector<uint32_t> nranges;        // rune mode: triples (lo, hi, cls), runes >= 0x80
  std::vector<uint8_t> cls_combo;       // multi: per class, bit0 '\n', bit1 word char
  std::vector<uint64_t> acc;            // multi: 5 masks per state
};

// Unanchored boolean search DFA for `re` (MatchString semantics).
bool build_regex_dfa(const Regex& re, Dfa* out, std::string* err, uint32_t state_cap = 60000);

// Union (multi-pattern) search DFA over up to 64 patterns: the scan reports,
// for every pattern, whether it matches somewhere in the input.
// byte_budget (0: none): the union is abandoned as soon as its states could no
// longer fit that many table bytes (2 B per transition + 8 B of accept masks
// per state) -- a failing trial stops early instead of running to state_cap.
bool build_union_dfa(const std::vector<const Regex*>& pats, Dfa* out, std::string* err,
                     uint32_t state_cap = 8192, uint32_t byte_budget = 0);

// @pm phrase set / @contains literal as a regex AST (search semantics).
// fold_ascii: ASCII-only case folding (aho-corasick AsciiCaseInsensitive).
// Returns false if a phrase has a byte >= 0x80 (byte-mode automaton needed).
bool phrases_to_regex(const std::vector<std::string>& phrases, bool fold_ascii, Regex* out);

// Aho-Corasick phrase automaton as a byte DFA: matches iff any phrase occurs.
// fold_ascii: ASCII case-insensitive (coraza @pm).
bool build_phrase_dfa(const std::vector<std::string>& phrases, bool fold_ascii, Dfa* out,
                      std::string* err, uint32_t state_cap = 60000);

// Exact matcher tables for a regex whose DFA exceeds the state cap: the
// Thompson NFA's class positions as bitsets (bit n_pos = match).
//   cm[c * words ..]                positions whose class holds rune class c
//   follow[(p * 16 + combo) * words] positions reachable after position p
//                                    (row n_pos: from the start) through epsilon
//                                    moves whose assertions hold for combo =
//                                    prev * 4 + next, prev / next in {0 none,
//                                    1 '\n', 2 word char, 3 other}
struct NfaTables {
  uint32_t n_classes = 0, n_pos = 0, words = 0;
  std::vector<uint8_t> amap;        // 128
  std::vector<uint32_t> nranges;    // (lo, hi, cls) for runes >= 0x80
  std::vector<uint8_t> cls_combo;   // bit0 '\n', bit1 word char
  std::vector<uint64_t> cm;
  std::vector<uint64_t> follow;
};
bool build_nfa_tables(const Regex& re, NfaTables* out, std::string* err, uint32_t max_pos = 4096);
bool nfa_host_match(const NfaTables& t, const uint8_t* s, size_t n);

// Pike VM program for submatch extraction (pike.h / pike.cpp), appended to
// insts / pool; false if it would exceed max_inst instructions.
struct DPikeInst;
struct DPike;
bool build_pike(const Regex& re, std::vector<DPikeInst>* insts, std::vector<uint32_t>* pool, DPike* out,
                std::string* err, uint32_t max_inst = 4096);

// Superset relaxation (level 1..3) for phase-A prefilter automata; see dfa.cpp.
void relax_regex(Regex* re, int level);

// Host-side walk of a built DFA (compiler self-test only; never used by the
// inspection path).
bool dfa_host_match(const Dfa& d, const uint8_t* s, size_t n);
// Multi automata: the set of patterns matching somewhere in s.
uint64_t dfa_host_scan(const Dfa& d, const uint8_t* s, size_t n);

// Go utf8.DecodeRune: returns rune, sets *w (invalid -> U+FFFD, width 1).
uint32_t go_decode_rune(const uint8_t* s, size_t n, size_t i, int* w);

}  // namespace gi
