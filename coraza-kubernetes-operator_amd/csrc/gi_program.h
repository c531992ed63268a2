// Device-resident rule program (the "GPU artifact" a RuleSet compiles to).
//
// Host (compile.cpp) builds these POD arrays once per RuleSet; the context
// uploads them to HBM and the inspection kernels interpret them.  Layout
// decisions are MI355X-first: everything a wavefront walks per byte (DFA
// transition rows, class maps) is in dense u16/u8 arrays; per-rule metadata
// is 64-byte aligned records read once per rule per request.
#pragma once
#include <stdint.h>

#include "pike.h"

#if !defined(__HIPCC__) && !defined(__host__)
#define __host__
#define __device__
#endif

// The per-request interpreter (kernels.hip: collect, transformations,
// operators, body processors, rule walk) is compiled for the GPU and, once
// more, for the host: gi_cpu_baseline_inspect runs the same code on the CPU
// cores as SURVEY §8(d)'s CPU baseline.  GI_HD marks that code; GI_TABLE its
// read-only tables (the GPU's constant memory; plain const arrays on the host).
#define GI_HD __host__ __device__
#if defined(__HIP_DEVICE_COMPILE__)
#define GI_TABLE __device__ __constant__
#else
#define GI_TABLE static const
#endif

namespace gi {

// Program records are immutable for the life of a context: reading them
// through the constant address space lets the compiler use scalar loads for
// wave-uniform indices (rule walk, operators, actions).
#if defined(__HIP_DEVICE_COMPILE__)
#define GI_CONST(T, p) ((const __attribute__((address_space(4))) T*)(p))
// copy record i of array p (sizeof(T) % 4 == 0) through the constant space
template <class T>
GI_HD __forceinline__ T gi_cload(const T* p, uint64_t i) {
  static_assert(sizeof(T) % 4 == 0, "record size");
  const __attribute__((address_space(4))) uint32_t* q =
      (const __attribute__((address_space(4))) uint32_t*)(p + i);
  uint32_t w[sizeof(T) / 4];
#pragma unroll
  for (uint32_t k = 0; k < sizeof(T) / 4; k++) w[k] = q[k];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}
#else
#define GI_CONST(T, p) ((const T*)(p))
template <class T>
GI_HD inline T gi_cload(const T* p, uint64_t i) {
  return p[i];
}
#endif

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
  S_REMOTE_ADDR,   // ProcessConnection
  S_REMOTE_PORT,
  S_FILES_COMBINED_SIZE,  // multipart: total part bytes
  S_ARGS_COMBINED_SIZE,   // computed when read: sum of key + value lengths of ARGS_GET and ARGS_POST
  S_FULL_REQUEST_LENGTH,  // declared, never set by coraza v3.3.3: ""
  S_URLENCODED_ERROR,     // declared, never set by coraza v3.3.3: ""
  S_INBOUND_DATA_ERROR,   // "1" when the body reached SecRequestBodyLimit
  S_SERVER_NAME,          // Transaction.SetServerName (gi_request.server_name; "" when not set)
  S_COUNT
};
#define GI_REQHDR_BYTES 384
#define GI_RM_BYTES 384  // per request: 8 ctl:ruleRemoveById ranges (128 B) + 8 ctl:ruleRemoveTargetById entries (32 B)  // per-request header slot (ReqHdr, kernels.hip) at the start of its scratch region

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
  V_XML,  // XML body processor output (kernels.hip parse_xml): FK_XML fields
  // MULTIPART body processor output (kernels.hip parse_multipart)
  V_FILES,                   // ("", file name) per file part
  V_FILES_NAMES,             // ("", part name) per file part
  V_FILES_SIZES,             // (file name, size) -- SetIndex per file name
  V_FILES_TMPNAMES,          // never populated (no upload storage, as coraza without a filesystem)
  V_MULTIPART_PART_HEADERS,  // (part name, "Key: value") per part header
  // matched-variable state of the transaction (coraza tx.matchVariable):
  // MATCHED_VAR / MATCHED_VAR_NAME persist across rules, MATCHED_VARS(_NAMES)
  // are reset before every top-level rule (RuleGroup.Eval)
  V_MATCHED_VAR,
  V_MATCHED_VAR_NAME,
  V_MATCHED_VARS,
  V_MATCHED_VARS_NAMES,
};

// Collection field kinds emitted by the collect stage.
enum FieldKind : uint8_t {
  FK_ARG_GET = 1, FK_ARG_POST = 2, FK_HEADER = 3, FK_COOKIE = 4,
  // multipart collections (after the phase-1 fields, among the ARGS_POST ones;
  // never phase-A items)
  FK_FILE = 5, FK_FILE_NAME = 6, FK_FILE_SIZE = 7, FK_PART_HEADER = 8,
  // XML body processor output: key "//@*" (attribute values) or "/*" (text)
  FK_XML = 9
};

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
  OP_IPMATCH,  // @ipMatch / @ipMatchFromFile: DOp.lit_off/lit_len = GI_IPNET_BYTES records in strpool
  OP_DETECT_SQLI,  // @detectSQLi (libinj.h; phase A: a DScanVal kind, evaluated in k_stream)
  OP_DETECT_XSS,   // @detectXSS
};
// @ipMatch network record (strpool, byte-addressed): [0] 4 = IPv4, 16 = IPv6;
// [1] prefix bits; [2..18) network address (IPv4 in bytes 2..6)
#define GI_IPNET_BYTES 18

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
  // out-of-line group (kernels.hip t_ext): decoders / encoders / digests
  T_BASE64DECODE,
  T_BASE64DECODEEXT,
  T_BASE64ENCODE,
  T_HEXDECODE,
  T_HEXENCODE,
  T_SHA1,
  T_MD5,
  T_URLENCODE,
  T_CSSDECODE,
  T_ESCAPESEQDECODE,
  T_REMOVECOMMENTSCHAR,
  T_COUNT
};

// D_ALLOW_*: the allow action [upstream internal/actions/allow.go]: "allow" (every remaining phase but
// logging), "allow:phase" (the rest of the current phase), "allow:request" (the rest of the request phases)
enum Disruptive : uint8_t {
  D_NONE = 0, D_DENY = 1, D_DROP = 2, D_REDIRECT = 3, D_PASS = 4,
  D_ALLOW_ALL = 5, D_ALLOW_PHASE = 6, D_ALLOW_REQUEST = 7
};

enum RuleFlags : uint8_t {
  RF_FOLDED = 128,  // first rule of a run of folded request-independent phase-1 rules: k_eval emits the
                    // run's matched ids and jumps past it (DRule._pad2 = run index, DProgram.fold_runs)
  RF_CONST = 64,  // request-independent link whose inputs are folded constants (compile.cpp fold_program):
                  // it matches DRule._pad2 values, whatever the request -- k_eval skips targets and operator
  RF_CHILD = 1,
  RF_MARKER = 2,
  RF_CAPTURE = 4,
  RF_BODYDEP = 8,  // targets can see ARGS_POST: phase-A bits ignored once a body was parsed
  RF_RESIDUAL = 16,  // some targets are residual (DVarRef.residual): a clear bit still tests them
  RF_MULTIMATCH = 32,  // multiMatch: the operator runs on the value and after every transformation
};

enum RuleFlags2 : uint8_t {
  RF2_MVS = 1,  // a later link of this chain reads MATCHED_VARS(_NAMES): k_eval keeps the entries
  RF2_MVCUR = 2,  // MATCHED_VAR / MATCHED_VAR_NAME this chain's matches set can be read (compile.cpp fold_program)
                // (otherwise only MATCHED_VAR / MATCHED_VAR_NAME are updated per match)
  RF2_BODY_PA = 4,  // a link of the chain runs an automaton / libinjection operator (@rx @pm @contains
                    // @containsWord @detectSQLi @detectXSS) over a body field collection: the gate's
                    // first stage (kernels.hip launch_pipeline) stops the phase-2 walk here until
                    // phase A has scanned the request's body fields
  RF2_PREFIX = 8,   // (any link) a link of a phase-2 rule before the first RF2_BODY_PA rule: its phase-A
                    // streams are "prefix" streams (DStream.prefix), which the gate's first stage runs over
                    // the body fields too -- its hit bits are complete there
  RF2_PA_RELAXED = 16,  // the link's phase-A automaton is a superset relaxation (its exact DFA exceeds the state
                        // cap): a phase-A hit is never an exact per-value match (k_eval re-runs the operator)
  RF2_PA_FILTER = 32,   // (first link) the phase-A pattern is a filter stronger than the operator (compile.cpp
                        // within_chain_filters): a value outside it has no effect but its capture record, so
                        // with capture records on k_eval visits the link and records those values' captures only
                        // (the link captures the whole value through t:lowercase: recorded inline)
  RF2_RESID_COLL = 64,  // RF_RESIDUAL only through body collections phase A does not scan (XML, part headers,
                        // FILES_TMPNAMES): empty -- so a clear bit is final -- unless the request's body went
                        // through the XML or multipart processor
  RF2_RESID_RB = 128,   // RF_RESIDUAL through REQUEST_BODY (and maybe body collections) only, and the link's
                        // chain + operator reject "": a clear bit is final while REQUEST_BODY is empty (and no
                        // XML / multipart body)
};

enum ActKind : uint8_t {
  A_SETVAR = 1,
  A_SETVAR_DEL,
  A_CTL_RULE_REMOVE_ID,
  A_CTL_RULE_ENGINE,
  A_CTL_BODY_PROCESSOR,
  A_CTL_BODY_ACCESS,
  A_CTL_FORCE_BODY,
  A_CTL_RULE_REMOVE_TARGET,  // ctl:ruleRemoveTargetById: a..b ids, slot = VarId, tmpl/_pad2 = key (strpool, lowercase);
                             // ctl:ruleRemoveTargetByTag / ByMsg: a = GI_RM_GROUP_MODE, b = the group's bit
  A_CTL_RULE_REMOVE_GROUP,   // ctl:ruleRemoveByTag / ruleRemoveByMsg: a = the group's bit (DProgram.rule_groups)
};
// ctl:ruleRemove*ByTag / ByMsg [upstream internal/actions/ctl.go]: the rules whose tags contain the value
// (whose msg equals it) are a "removal group" fixed at compile time; a request's removed groups are a
// 32-bit mask tested against DProgram.rule_groups[rule index]
#define GI_MAX_RM_GROUPS 32
#define GI_RM_GROUP_MODE INT64_MIN

// setvar fast forms (DAction.a for A_SETVAR)
enum SetvarForm : int64_t {
  SV_GENERIC = 0,
  SV_SET_INT = 1,    // =<canonical integer literal b>
  SV_ADD_CONST = 2,  // =+<integer literal b>
  SV_SUB_CONST = 3,  // =-<integer literal b>
  SV_ADD_SLOT = 4,   // =+%{tx.<slot b>}
  SV_SUB_SLOT = 5,   // =-%{tx.<slot b>}
};

enum EngineMode : uint8_t { ENGINE_OFF = 0, ENGINE_ON = 1, ENGINE_DETECTION_ONLY = 2 };
enum BodyProc : uint8_t { BP_NONE = 0, BP_URLENCODED = 1, BP_JSON = 2, BP_XML = 3, BP_MULTIPART = 4 };

enum TPartKind : uint8_t { TP_LIT = 1, TP_TX, TP_SINGLE, TP_HEADER, TP_MV, TP_MVNAME };

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
  uint8_t flags2;       // RF2_* (top-level rules)
  int32_t hit_slot;     // phase-A hit bit (-1: evaluated by the interpreter only)
  uint32_t _pad2;       // RF_CONST: the number of values the link matches (its actions run that often);
                        // RF_FOLDED: its run
};

// Folded TX state after the request-independent prefix of phase 1 (compile.cpp
// fold_program): one record per TX slot, state as in kernels.hip Slot (0 unset,
// 1 integer num, 2 string strpool[off, off + len)).  The runtime turns it into
// device Slot records; k_eval reads a slot from it until the request writes
// the slot (copy on write).
struct DSnapSlot {
  int64_t num;
  uint32_t off, len;
  uint32_t state, _pad;
};

// ------------------------------------------------------ phase-A scan plan
// stream  = one transformation chain: every value some target of a phase-A
//           rule link reads through that chain.  k_stream transforms each
//           admitted value ONCE per stream into the request's phase-A arena;
// filter  = one value source of the stream: a single variable, or a field
//           kind set (key or value side) with a key selector + exclusions;
// pattern = one phase-A-eligible rule link on the stream, admitted by the
//           filters of its targets; a value feeds a pattern only through
//           one of those filters;
// job     = up to GI_JOB_MAX_DFA automata of one stream whose tables fit one
//           LDS image: a persistent k_scan workgroup loads the image once and
//           sweeps the stream's arena segment of many requests, stepping the
//           job's automata in lockstep over each value.
#define GI_MAX_FILTERS 32
#define GI_MAX_STREAMS 256  // streams a ruleset may have (k_stream keeps per-stream chunk state in LDS)
#define GI_MAX_GFILTERS 64
#define GI_JOB_LDS_BYTES 65536          // small jobs: 2 workgroups of 1024 per CU
#define GI_BIG_LDS_BYTES (148 * 1024)   // big jobs: 1 workgroup of 1024 per CU (+ 8 KB k_scan block list)
#define GI_JOB_MAX_DFA 4
#define GI_JAMAP_BYTES 1024             // joint class map: u32[256] (>= 0x80: rune-mapped non-ASCII), byte q = class in automaton q
#define GI_RUNE_MARK 0x80               // a non-ASCII rune in a collapsed value
#define GI_NO_SINGLE 0xFF

struct DStream {
  uint32_t tchain_off, tchain_len;
  uint32_t filt_begin, filt_count;  // DFilter
  uint32_t job_begin, job_count;    // DJob (contiguous per stream)
  uint32_t val_begin, val_count;    // DScanVal: validate operators, evaluated by k_stream
  uint64_t gmask;     // the stream's filters as global filter ids
  uint8_t kind_mask;  // union of the field filters' kinds (1 << FieldKind)
  uint8_t collapse;   // values are rune-mapped for the scan instead of slow: each non-ASCII rune
                      // becomes one byte, GI_RUNE_MARK (rmap_cnt 0: the automata agree on all of
                      // them) or 0x80 + its joint class (rmap triples (lo, hi, byte) in nranges)
  uint8_t det_id;     // index in DProgram.det_streams if some val is @detectSQLi/@detectXSS, else 0xFF
  uint8_t prefix;     // some job / value test of it is DJob.prefix / DScanVal.prefix: the gate's first stage
                      // runs body fields through its chain
  uint32_t rmap_off, rmap_cnt;
  uint32_t _pad2;
};
#define GI_MAX_DET_STREAMS 32

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
  uint32_t key_hash;  // gi_fnv1a of the literal key (as stored: lowercase when ci)
};

// FNV-1a over bytes (key prefilter of the phase-A filters; host and device).
__host__ __device__ inline uint32_t gi_fnv1a(const uint8_t* s, uint32_t n, bool lower) {
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t c = s[i];
    if (lower && c >= 'A' && c <= 'Z') c += 32;
    h = (h ^ c) * 16777619u;
  }
  return h;
}

// Byte summary of a value: which bytes that make some transformation
// non-identity occur in it.  A transformation whose trigger set does not meet
// the summary leaves the value unchanged, so it is skipped outright (exact).
enum : uint32_t {
  BS_PCT = 1u << 0, BS_PLUS = 1u << 1, BS_AMP = 1u << 2, BS_UPPER = 1u << 3, BS_HIGH = 1u << 4,
  BS_NUL = 1u << 5, BS_WS = 1u << 6, BS_SLASH = 1u << 7, BS_BSLASH = 1u << 8, BS_DOT = 1u << 9,
  BS_QUOTE = 1u << 10, BS_CARET = 1u << 11, BS_SEP = 1u << 12, BS_ALL = 0xFFFFFFFFu,
  // k_stream's summary LUT only: a byte outside [A-Za-z0-9_] / a byte of the
  // XSS trigger set (libinj.h li_sqli_byte / li_xss_byte; no transformation triggers on them)
  BS_LI_SQLI = 1u << 13, BS_LI_XSS = 1u << 14,
};
__host__ __device__ inline uint32_t byte_summary(uint8_t c) {
  uint32_t m = 0;
  m |= c == '%' ? BS_PCT : 0u;
  m |= c == '+' ? BS_PLUS : 0u;
  m |= c == '&' ? BS_AMP : 0u;
  m |= (c >= 'A' && c <= 'Z') ? BS_UPPER : 0u;
  m |= c >= 0x80 ? BS_HIGH : 0u;
  m |= c == 0 ? BS_NUL : 0u;
  m |= (c == ' ' || (c >= 9 && c <= 13)) ? BS_WS : 0u;
  m |= c == '/' ? BS_SLASH : 0u;
  m |= c == '\\' ? BS_BSLASH : 0u;
  m |= c == '.' ? BS_DOT : 0u;
  m |= (c == '"' || c == '\'') ? BS_QUOTE : 0u;
  m |= c == '^' ? BS_CARET : 0u;
  m |= (c == ',' || c == ';') ? BS_SEP : 0u;
  return m;
}
// Bytes that can make transformation `code` change its input
// ([upstream] internal/transformations/*.go, restated above).
__host__ __device__ inline uint32_t transform_triggers(uint8_t code) {
  switch (code) {
    case T_LOWERCASE: return BS_UPPER | BS_HIGH;
    case T_URLDECODE:
    case T_URLDECODEUNI: return BS_PCT | BS_PLUS;
    case T_HTMLENTITYDECODE: return BS_AMP;
    case T_REMOVENULLS:
    case T_REPLACENULLS: return BS_NUL;
    case T_REMOVEWHITESPACE:
    case T_COMPRESSWHITESPACE:
    case T_TRIM:
    case T_TRIMLEFT:
    case T_TRIMRIGHT: return BS_WS | BS_HIGH;
    case T_REPLACECOMMENTS: return BS_SLASH;
    case T_CMDLINE: return BS_QUOTE | BS_BSLASH | BS_CARET | BS_WS | BS_SEP | BS_UPPER;
    case T_NORMALIZEPATH: return BS_SLASH | BS_DOT;
    case T_NORMALIZEPATHWIN: return BS_SLASH | BS_DOT | BS_BSLASH;
    case T_JSDECODE:
    case T_CSSDECODE:
    case T_ESCAPESEQDECODE: return BS_BSLASH;
    case T_UTF8TOUNICODE: return BS_HIGH;
    default: return BS_ALL;  // t:length and anything new: always run
  }
}

// Transformation `code` leaves a value with byte summary `summ` unchanged: its
// trigger set misses the summary.  BS_ALL marks transformations that must
// always run (t:length, encoders, digests): never an identity, even on a value
// whose summary is empty.
__host__ __device__ inline bool transform_identity(uint32_t summ, uint8_t code) {
  const uint32_t tr = transform_triggers(code);
  return tr != BS_ALL && !(summ & tr);
}

// Image of an LDS job (byte offsets inside the job's image):
//   [0, 512)      joint ASCII class map (u32 per byte < 0x80)
//   per automaton: transitions u16[n_states][n_classes] (state index, bit 15 =
//                  accepting transition of a union automaton; the absorbing
//                  accept row of a single automaton loops to itself),
//                  class map (128 rune-mode / 256 byte-mode), combo (union),
//                  end-of-input accept (u8 per state single / u64 per state union)
//   fmask         u64[jdfa_count][n_gfilters]: patterns each (global) filter admits
//   slots         u32 hit slot per pattern, automata concatenated
struct DJob {
  uint32_t stream;
  uint32_t img_off, img_bytes;     // LDS image (u8 image pool, 16-B aligned)
  uint32_t jdfa_begin, jdfa_count; // DJobDfa
  uint32_t lds_fmask;              // image offset of the fmask table
  uint8_t lds;                     // 1: all automata in the image; 0: one automaton on global tables
  uint8_t big;                     // image > GI_JOB_LDS_BYTES (big-LDS launch)
  uint8_t prefix;                  // a RF2_PREFIX link's pattern is in it: the gate's first stage runs it over
                                   // body fields (the body stage the others)
  uint8_t _pad;
};

struct DJobDfa {
  int32_t dfa;        // DDfa (start, classes, accept masks, rune ranges)
  int32_t lds_trans;  // image offsets (lds jobs), -1 otherwise
  int32_t lds_amap;
  int32_t lds_combo;
  int32_t lds_endacc;
  int32_t lds_slots;  // u32 hit slot per pattern
  uint32_t pat_begin; // DPat, n_pat entries (bit k of the match mask)
  uint32_t n_pat;
  uint32_t fmask_off; // u64 pool: per global filter, the patterns it admits
  uint32_t _pad;
  uint64_t neg_mask;  // patterns whose operator is negated
};

struct DPat {
  uint32_t slot;      // hit slot of the rule link
};

struct DScanVal {     // @validateByteRange / @validateUrlEncoding / @validateUtf8Encoding / @detectSQLi / @detectXSS
  uint8_t kind;
  uint8_t negate;
  uint8_t prefix;     // a RF2_PREFIX link's value test (as DJob.prefix)
  uint8_t _pad;
  uint32_t slot;
  uint64_t fmask;     // admitting filters (global filter ids)
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
  int32_t slot;      // TX literal key -> slot (TX regex key: key_off / key_len = the static slots it
                     // matches in DProgram.txrx; dynamic keys are matched at run time)
  uint8_t residual;  // a body-phase single (REQUEST_BODY, ...) of a phase-A link: phase A does
                     // not see it, so a clear hit bit leaves it for k_eval to test
  uint8_t pre_len;   // TX regex key of the form ^<literal>: the literal's length (slot = its strpool
                     // offset): run-time keys are matched by a prefix compare instead of the automaton
  uint8_t _pad[2];
};

struct DExc {
  int32_t dfa;       // regex exception (matched on the lowercased key) or -1
  uint32_t off, len; // literal exception (lowercase)
  uint32_t hash;     // gi_fnv1a of the literal exception
};

struct DOp {
  uint8_t kind;
  uint8_t negate;
  uint8_t arg_is_lit;  // template is a single literal (no macro)
  uint8_t has_num;     // literal numeric arg parsed at compile time (Atoi ok)
  int32_t dfa;
  int32_t nfa;         // @rx whose DFA exceeds the state cap: exact NFA tables (DNfa), else -1
  int32_t tmpl;
  uint32_t lit_off, lit_len;
  uint32_t ngroups;    // @pm / @pmFromFile over a large phrase set: automata dfa .. dfa + ngroups - 1
                       // (phrase groups, any match), else 0
  int32_t pike;        // @rx of a link whose `capture` is observable: submatch program (DPike), else -1
  int64_t num;
  uint32_t bits[8];    // @validateByteRange allowed-byte bitmap
};

// Exact matcher of an @rx whose DFA exceeds the state cap (regex.h
// NfaTables): position bitsets of `words` u64 each, bit n_pos = match.
#define GI_NFA_MAX_WORDS 64  // 4095 positions
struct DNfa {
  uint32_t n_classes, n_pos, words, nr_cnt;
  uint32_t amap_off;    // u8 pool: 128 ASCII classes
  uint32_t combo_off;   // u8 pool: per class bit0 '\n', bit1 word char
  uint32_t nr_off;      // u32 pool (nranges): (lo, hi, cls) triples
  uint32_t _pad;
  uint64_t cm_off;      // u64 pool: [n_classes][words]
  uint64_t follow_off;  // u64 pool: [n_pos + 1][16][words]
};

struct DAction {
  uint8_t kind;
  uint8_t _pad[3];
  int32_t slot;   // A_SETVAR*: TX slot; -1: the key has a macro (aux = its template, see DDynSite)
  int32_t tmpl;   // A_SETVAR: value template (-1: empty value)
  int32_t aux;    // A_SETVAR* with slot -1: key template; A_CTL_RULE_REMOVE_TARGET: key length
  int64_t a, b;   // ctl arguments
};

// A setvar whose key has a macro (setvar:'tx.header_name_920450_%{tx.0}=...')
// creates TX keys at run time: k_eval keeps them in the request's dynamic TX
// area (DynHdr + DynEnt[cap] + bytes, kernels.hip dyn_slot).  One record per
// such action, for the host to size that area from the request (runtime.cpp):
//   executions <= mm * (nsingles + (hdr_names + hdr_vals) * headers + other_coll * field capacity),
//                 (each a count of such targets)
//                 or mm when the rule has no targets (SecAction)
//   bytes      <= executions * (lit + fixed + 32 * n_mvname)
//                 + g * (n_val + n_mvname) * (bytes of the values the targets can produce)
//                 + executions * n_big * max(cap_t, cap_mt)
// where g is g_ascii when those bytes are ASCII, else g_any (the growth of the
// link's transformation chain: the matched value a %{tx.<digit>} capture,
// %{MATCHED_VAR} or %{MATCHED_VAR_NAME} part reads is at most g x its raw bytes).
struct DDynSite {
  uint32_t mm;         // multiMatch: transformations + 1, else 1
  uint32_t lit;        // literal bytes of the key and value templates
  uint32_t fixed;      // bytes per execution a digest / length transformation may yield
  uint32_t nsingles;   // single-variable targets
  uint32_t n_val;      // parts reading the matched value (own capture group, MATCHED_VAR)
  uint32_t n_mvname;   // MATCHED_VAR_NAME parts
  uint32_t n_big;      // other macro parts (any TX value, singles, headers): <= max(cap_t, cap_mt) each
  uint32_t g_ascii, g_any;
  uint8_t hdr_names, hdr_vals, other_coll;  // targets: REQUEST_HEADERS_NAMES, REQUEST_HEADERS, other collections
  uint8_t no_targets;
  uint32_t prefix_off, prefix_len;  // the key template's leading literal (strpool, lowercase)
  uint32_t dead;                    // the rule is unreachable (behind a constant gate): no area for it
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
  const uint32_t* tchains32;    // the same codes widened (scalar-loadable in wave-uniform loops)
  const DDfa* dfas;
  const DNfa* nfas;
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
  const uint32_t* sfilt;        // per stream filter: global filter id (filters[] is global)
  const uint32_t* always_slots; // hit slots without an automaton image
  const uint32_t* body_links;   // links k_body tests on the speculative REQUEST_BODY
  const DPike* pikes;           // submatch programs of observable captures (pike.h)
  const DPikeInst* pike_insts;
  const uint32_t* pike_ranges;
  uint32_t cap_ws_words;        // pike_match workspace per request (max over the programs; 0: none)
  uint32_t cap_groups;          // capture groups written at most (TX.0 .. TX.<cap_groups - 1>)
  int32_t cap_slots[9];         // TX slot of the keys "0".."8" (capture targets), -1 when none
  uint32_t n_body_links;
  uint32_t n_always;
  uint32_t n_gfilters;
  uint32_t item_singles;        // singles some filter reads (1 << SingleId)
  uint8_t item_sides[8];        // per FieldKind: bit0 value side, bit1 key side
  uint32_t n_jobs;
  uint32_t n_hit_slots;
  uint32_t max_img_bytes;       // largest small-job image
  uint32_t max_big_img_bytes;   // largest big-job image (0: none)
  uint32_t n_streams;
  uint32_t n_lower_pairs;
  uint32_t n_top;
  uint32_t top_begin[2], top_end[2];  // per-phase walks in top[] (phase 1, phase 2)
  const uint32_t* top_jump;           // per walk entry: where its rule's skipAfter resumes (runtime.cpp)
  const uint32_t* slot_hash;          // static TX slot by name: open addressing on gi_fnv1a, entry = slot + 1
  uint32_t slot_hash_mask;            // (runtime.cpp; a macro-key setvar resolves to a static slot first)
  uint32_t n_dyn_sites;               // macro-key setvars (DDynSite): requests carry a dynamic TX area
  const uint32_t* txrx;               // static slots a regex-keyed TX target matches (DVarRef.key_off/len)
  // request-independent phase-1 rules, evaluated at compile time (fold_program):
  const uint8_t* tx_snap;             // Slot[n_slots] (kernels.hip) after it
  const uint32_t* fold_ids;           // the ids the folded rules matched, in walk order
  const uint32_t* fold_runs;          // per run: ids offset, count, walk index after it, pending skipAfter
  uint32_t fold_nids;
  uint32_t fold_on;                   // 0: nothing folded (TX starts empty)
  uint32_t n_slots;
  uint32_t n_markers;
  int32_t exports[8];           // TX slot per export, -1 = none
  uint32_t n_exports;
  uint32_t hist_mask;           // exports whose sum the score histogram bins (runtime.cpp: the per-paranoia-level
                                // inbound scores when exported, else export 0)
  uint8_t rule_engine;          // EngineMode
  uint8_t body_access;
  uint8_t mv_used;              // some target / macro reads MATCHED_VAR(S)(_NAME(S)): k_eval records matches
  uint8_t body_partial;         // SecRequestBodyLimitAction ProcessPartial (else Reject)
  uint64_t body_limit;
  const uint32_t* rule_groups;  // per rule record: the ctl removal groups (ByTag / ByMsg) it belongs to
  uint32_t n_rm_groups;         // 0: no ctl:ruleRemove*ByTag / ByMsg in the program
  uint32_t args_limit;          // SecArgumentsLimit (coraza WAF.ArgumentLimit, default 1000): ARGS_GET
  uint32_t n_det_streams;       // streams with @detectSQLi/@detectXSS vals (k_detect entries carry a mask)
  uint32_t det_streams[GI_MAX_DET_STREAMS];
};

}  // namespace gi
