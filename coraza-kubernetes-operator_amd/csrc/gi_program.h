// Device-resident rule program (the "GPU artifact" a RuleSet compiles to).
//
// Host (compile.cpp) builds these POD arrays once per RuleSet; the context
// uploads them to HBM and the inspection kernels interpret them.  Layout
// decisions are MI355X-first: everything a wavefront walks per byte (DFA
// transition rows, class maps) is in dense u16/u8 arrays; per-rule metadata
// is 64-byte aligned records read once per rule per request.
#pragma once
#include <stdint.h>

namespace gi {

// ------------------------------------------------------------- variables
// Scalar variables ("collection.Single" in coraza) -- per-request table index.
enum SingleId : uint8_t {
  S_REQUEST_METHOD = 0,
  S_REQUEST_PROTOCOL,
  S_REQUEST_URI,
  S_REQUEST_URI_RAW,
  S_REQUEST_LINE,
  S_REQUEST_FILENAME,
  S_REQUEST_BASENAME,
  S_QUERY_STRING,
  S_REQUEST_BODY,
  S_REQUEST_BODY_LENGTH,
  S_REQBODY_ERROR,
  S_REQBODY_ERROR_MSG,
  S_REQBODY_PROCESSOR,
  S_MULTIPART_STRICT_ERROR,
  S_COUNT
};

// Variable ids used by rule targets.  [0, S_COUNT) are singles.
enum VarId : uint8_t {
  V_ARGS_GET = 32,
  V_ARGS_POST,
  V_ARGS,
  V_REQUEST_HEADERS,
  V_REQUEST_COOKIES,
  V_TX,
  V_ARGS_GET_NAMES,
  V_ARGS_POST_NAMES,
  V_ARGS_NAMES,
  V_REQUEST_HEADERS_NAMES,
  V_REQUEST_COOKIES_NAMES,
  V_XML,  // XML body processor output: never populated (XML bodies are flagged unsupported)
  V_FILES,        // multipart output: never populated (multipart bodies are flagged unsupported)
  V_FILES_NAMES,
};

// Collection field kinds emitted by the collect stage.
enum FieldKind : uint8_t { FK_ARG_GET = 1, FK_ARG_POST = 2, FK_HEADER = 3, FK_COOKIE = 4 };

// ------------------------------------------------------------- operators
enum OpKind : uint8_t {
  OP_RX = 1,
  OP_PM,
  OP_CONTAINS,
  OP_CONTAINSWORD,
  OP_STREQ,
  OP_BEGINSWITH,
  OP_ENDSWITH,
  OP_WITHIN,
  OP_EQ,
  OP_GE,
  OP_GT,
  OP_LE,
  OP_LT,
  OP_UNCONDITIONAL,
  OP_NOMATCH,
  OP_VALIDATE_BYTE_RANGE,
  OP_VALIDATE_URL_ENCODING,
  OP_VALIDATE_UTF8,
};

// --------------------------------------------------------- transformations
enum TCode : uint8_t {
  T_LOWERCASE = 1,
  T_URLDECODE,
  T_URLDECODEUNI,
  T_HTMLENTITYDECODE,
  T_REMOVENULLS,
  T_REPLACENULLS,
  T_REMOVEWHITESPACE,
  T_COMPRESSWHITESPACE,
  T_REPLACECOMMENTS,
  T_CMDLINE,
  T_LENGTH,
  T_TRIM,
  T_TRIMLEFT,
  T_TRIMRIGHT,
  T_NORMALIZEPATH,
  T_NORMALIZEPATHWIN,
  T_JSDECODE,
  T_UTF8TOUNICODE,
};

enum Disruptive : uint8_t { D_NONE = 0, D_DENY = 1, D_DROP = 2, D_REDIRECT = 3, D_PASS = 4 };

enum RuleFlags : uint8_t {
  RF_CHILD = 1,
  RF_MARKER = 2,
  RF_CAPTURE = 4,
  RF_BODYDEP = 8,  // targets can see ARGS_POST: phase-A bits ignored once a body was parsed
};

enum ActKind : uint8_t {
  A_SETVAR = 1,
  A_SETVAR_DEL,
  A_CTL_RULE_REMOVE_ID,
  A_CTL_RULE_ENGINE,
  A_CTL_BODY_PROCESSOR,
  A_CTL_BODY_ACCESS,
  A_CTL_FORCE_BODY,
};

enum EngineMode : uint8_t { ENGINE_OFF = 0, ENGINE_ON = 1, ENGINE_DETECTION_ONLY = 2 };
enum BodyProc : uint8_t { BP_NONE = 0, BP_URLENCODED = 1, BP_JSON = 2, BP_XML = 3, BP_MULTIPART = 4 };

enum TPartKind : uint8_t { TP_LIT = 1, TP_TX, TP_SINGLE, TP_HEADER };

// ---------------------------------------------------------------- records
struct DRule {
  int32_t id;
  int32_t status;
  int32_t skip;
  int32_t chain_next;   // next chain link (rule index) or -1
  int32_t skip_after;   // marker id or -1
  int32_t marker;       // marker id if this is a SecMarker, else -1
  uint32_t var_begin, var_count;
  int32_t op;           // op index, -1 = no operator (SecAction)
  uint32_t tchain_off, tchain_len;
  uint32_t act_begin, act_count;
  uint8_t phase;
  uint8_t disruptive;
  uint8_t flags;        // RuleFlags
  uint8_t _pad;
  int32_t hit_slot;     // phase-A hit bit (-1: evaluated by the interpreter only)
  uint32_t _pad2;
};

// ------------------------------------------------------ phase-A scan plan
// stream  = one transformation chain: every value some target of a phase-A
//           rule link reads through that chain (values are transformed once
//           per job and scanned by every automaton of the job);
// filter  = one value source of the stream: a single variable, or a field
//           kind set (key or value side) with a key selector + exclusions;
// pattern = one phase-A-eligible rule link on the stream, admitted by the
//           filters of its targets; a value feeds a pattern only through
//           one of those filters;
// job     = the automata of one stream whose tables fit one LDS image: a
//           persistent workgroup loads the image once and sweeps requests.
#define GI_MAX_FILTERS 32
#define GI_JOB_LDS_BYTES 65536
#define GI_NO_SINGLE 0xFF

struct DStream {
  uint32_t tchain_off, tchain_len;
  uint32_t filt_begin, filt_count;  // DFilter
  uint8_t kind_mask;  // union of the field filters' kinds (1 << FieldKind)
  uint8_t _pad[3];
};

struct DFilter {
  uint8_t single;     // SingleId, or GI_NO_SINGLE for a field filter
  uint8_t kind_mask;  // 1 << FieldKind
  uint8_t names;      // the key is the value
  uint8_t key_mode;   // 0 none, 1 literal, 2 regex
  uint8_t ci;         // case-insensitive keys
  uint8_t _pad[3];
  int32_t key_dfa;
  uint32_t key_off, key_len;
  uint32_t exc_begin, exc_count;
};

struct DJob {
  uint32_t stream;
  uint32_t img_off, img_bytes;     // LDS image (u8 image pool, 16-B aligned)
  uint32_t jdfa_begin, jdfa_count; // DJobDfa
  uint32_t val_begin, val_count;   // DScanVal
};

struct DJobDfa {
  int32_t dfa;        // DDfa (start, classes, accept masks, rune ranges)
  int32_t lds_trans;  // byte offset of the transition table in the image, -1: global
  int32_t lds_amap;   // byte offset of the 128/256-entry class map in the image
  int32_t lds_combo;  // byte offset of the per-class combo table (multi)
  uint32_t pat_begin; // DPat, n_pat entries (bit k of the match mask)
  uint32_t n_pat;
  uint32_t fmask_off; // u64 pool: per stream filter, the patterns it admits
  uint32_t _pad;
  uint64_t neg_mask;  // patterns whose operator is negated
};

struct DPat {
  uint32_t slot;      // hit slot of the rule link
};

struct DScanVal {     // @validateByteRange / @validateUrlEncoding / @validateUtf8Encoding
  uint8_t kind;
  uint8_t negate;
  uint8_t _pad[2];
  uint32_t fmask;     // admitting filters
  uint32_t slot;
  uint32_t _pad2;
  uint32_t bits[8];
};

struct DVarRef {
  uint8_t var;       // SingleId or VarId
  uint8_t count;     // &VAR
  uint8_t key_mode;  // 0 none, 1 literal, 2 regex
  uint8_t ci;        // case-insensitive keys (headers, TX)
  int32_t key_dfa;
  uint32_t key_off, key_len;  // literal key in string pool (lowercased when ci)
  uint32_t exc_begin, exc_count;
  int32_t slot;      // TX literal key -> slot
  uint32_t _pad;
};

struct DExc {
  int32_t dfa;       // regex exception (matched on the lowercased key) or -1
  uint32_t off, len; // literal exception (lowercase)
};

struct DOp {
  uint8_t kind;
  uint8_t negate;
  uint8_t arg_is_lit;  // template is a single literal (no macro)
  uint8_t has_num;     // literal numeric arg parsed at compile time (Atoi ok)
  int32_t dfa;
  int32_t tmpl;
  uint32_t lit_off, lit_len;
  int64_t num;
  uint32_t bits[8];    // @validateByteRange allowed-byte bitmap
};

struct DAction {
  uint8_t kind;
  uint8_t _pad[3];
  int32_t slot;   // A_SETVAR*: TX slot
  int32_t tmpl;   // A_SETVAR: value template (-1: empty value)
  int32_t _pad2;
  int64_t a, b;   // ctl arguments
};

struct DTmplPart {
  uint8_t kind;
  uint8_t single;
  uint16_t _pad;
  int32_t slot;
  uint32_t off, len;  // TP_LIT / TP_HEADER key (lowercase)
};

struct DTmpl {
  uint32_t part_begin, part_count;
};

struct DDfa {
  uint32_t n_states, n_classes, start, accept;
  uint32_t trans_off;    // u16 pool
  uint32_t endacc_off;   // u8 pool
  uint32_t amap_off;     // u8 pool (128 rune mode / 256 byte mode)
  uint32_t nr_off, nr_cnt;  // u32 pool triples (lo, hi, cls)
  uint8_t byte_mode;
  uint8_t nonascii_uniform;  // every rune >= 0x80 maps to nonascii_cls
  uint8_t nonascii_cls;
  uint8_t multi;             // union automaton (see regex.h)
  uint32_t combo_off;        // u8 pool: per-class combo (multi)
  uint32_t acc_off;          // u64 pool: 5 masks per state (multi)
};

// Everything the kernels need, as device pointers (filled by the context).
struct DProgram {
  const DRule* rules;
  const uint32_t* top;
  const DVarRef* vars;
  const DExc* excs;
  const DOp* ops;
  const DAction* acts;
  const DTmplPart* tparts;
  const DTmpl* tmpls;
  const uint8_t* tchains;
  const DDfa* dfas;
  const uint16_t* trans;
  const uint8_t* u8pool;
  const uint32_t* nranges;
  const uint8_t* strpool;
  const uint32_t* lower_pairs;  // unicode.ToLower table (rune, lower) pairs
  const uint32_t* slot_names;   // (off, len) into strpool per TX slot
  const uint64_t* u64pool;      // union-automaton accept masks
  const DStream* streams;
  const DFilter* filters;
  const DJob* jobs;
  const DJobDfa* jdfas;
  const DPat* pats;
  const DScanVal* svals;
  const uint8_t* images;        // LDS images of the jobs
  uint32_t n_jobs;
  uint32_t n_hit_slots;
  uint32_t max_img_bytes;
  uint32_t n_lower_pairs;
  uint32_t n_top;
  uint32_t n_slots;
  uint32_t n_markers;
  int32_t exports[8];           // TX slot per export, -1 = none
  uint32_t n_exports;
  uint8_t rule_engine;          // EngineMode
  uint8_t body_access;
  uint8_t _pad[2];
  uint64_t body_limit;
};

}  // namespace gi
