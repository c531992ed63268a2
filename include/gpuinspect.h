/*
 * gpuinspect -- MI355X-native batched WAF inspection engine (C ABI).
 *
 * Drop-in boundary for the Coraza Kubernetes Operator's rule-evaluation hot
 * path.  Each entry point names the reference interface it replaces:
 *
 *   gi_compile        coraza.NewWAF(coraza.NewWAFConfig().WithDirectives(s))
 *                     -- /root/reference/internal/controller/ruleset_controller.go:159-160
 *                     (compile/validate a RuleSet's SecLang; error text is
 *                     surfaced like the InvalidConfigMap status at :161-170).
 *                     The aggregated text it takes is RuleSetEntry.Rules
 *                     (internal/rulesets/cache/cache.go:32-36), the string the
 *                     data plane fetches from GET /rules/<key> (server.go:183-198).
 *   gi_inspect_batch  the per-request Coraza transaction the data plane
 *                     (coraza-proxy-wasm, config/samples/engine.yaml:12) runs:
 *                     NewTransaction -> ProcessURI -> AddRequestHeader* ->
 *                     ProcessRequestHeaders (phase 1) -> WriteRequestBody ->
 *                     ProcessRequestBody (phase 2) -> Interruption() /
 *                     MatchedRules() -> Close()   [coraza/v3 v3.3.3, go.mod:6]
 *                     -- for a whole batch of requests at once.
 *   gi_ruleset_free   (WAF values are garbage collected in Go)
 *
 * Ownership / threading: a gi_ruleset is immutable after gi_compile and may
 * be shared by any number of contexts/threads (like a coraza WAF).  A gi_ctx
 * owns device buffers and one HIP stream; one thread at a time per ctx (like
 * a coraza Transaction).  Input buffers are borrowed for the duration of a
 * call.  Errors are return codes, never exceptions across the ABI.
 *
 * There is no CPU evaluation path: every gi_inspect_* call runs the HIP
 * kernels on the ctx's device, and fails with GI_ENODEV without one.
 */
#ifndef GPUINSPECT_H
#define GPUINSPECT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- codes */
#define GI_OK 0
#define GI_EPARSE -1       /* SecLang syntax error (coraza.NewWAF error) */
#define GI_EUNSUPPORTED -2 /* valid SecLang this engine does not implement */
#define GI_EINVAL -3
#define GI_STATS_LAUNCHES 48 /* gi_stats per-launch records */
#define GI_ENODEV -4       /* no HIP device / kernel launch failure */
#define GI_ENOMEM -5
#define GI_ETRUNC -6       /* caller-provided result capacity too small */
#define GI_ESTATE -7       /* call order (e.g. run before stage) */

/* per-request verdict flags (gi_verdict.flags) */
#define GI_REQ_UNSUPPORTED_URI 0x1   /* request-target outside the supported forms */
#define GI_REQ_UNSUPPORTED_BODY 0x2  /* body processor not implemented, or a body beyond the engine's limits */
#define GI_REQ_BODY_LIMIT 0x4        /* (no longer set: an over-limit body gets coraza's 413 / ProcessPartial) */
#define GI_REQ_OVERFLOW 0x8          /* internal per-request capacity exceeded */
#define GI_REQ_MATCH_TRUNC 0x10      /* more matched rules than matched_cap */
#define GI_REQ_BODY_ERROR 0x20       /* the body processor rejected the body: REQBODY_ERROR=1 (verdict valid) */
#define GI_REQ_CAPTURE_TRUNC 0x40    /* more capture records / bytes than the ctx's capture caps (verdict valid) */
#define GI_REQ_ERROR_MASK 0x0F       /* verdict is not valid when any of these is set */

/* interruption action (coraza types.Interruption.Action) */
#define GI_ACTION_NONE 0
#define GI_ACTION_DENY 1
#define GI_ACTION_DROP 2
#define GI_ACTION_REDIRECT 3

#define GI_MAX_EXPORTS 8

typedef struct gi_ruleset gi_ruleset;
typedef struct gi_ctx gi_ctx;

typedef struct {
  /* TX variables whose final integer value is exported per request
   * (NULL-terminated list; NULL = default CRS anomaly-score set:
   * blocking_inbound_anomaly_score, inbound_anomaly_score_pl1..pl4,
   * detection_inbound_anomaly_score, anomaly_score, 0) */
  const char* const* tx_exports;
  uint32_t dfa_state_cap; /* 0 = default (60000) */
  /* @pmFromFile data files (coraza internal/operators/pm_from_file.go reads
   * them from disk; the reference build strips those rules because it is
   * built with no_fs_access, Makefile:43).  The caller passes each file the
   * rules name as (name, bytes); a rule naming a file not given here fails
   * with GI_EPARSE, like a missing file in Coraza. */
  uint32_t n_data_files;
  const char* const* data_file_names;
  const char* const* data_file_data;
  const size_t* data_file_lens;
} gi_compile_opts;

typedef struct {
  uint32_t n_rules;      /* top-level rules (SecRule/SecAction/SecMarker) */
  uint32_t n_links;      /* all rule records including chain links */
  uint32_t n_dfas;
  uint32_t n_tx_slots;
  uint64_t program_bytes; /* device-resident artifact size */
  uint32_t n_scan_jobs;   /* phase-A jobs (one LDS-resident automaton image each) */
  uint32_t n_hit_slots;   /* rule links evaluated data-parallel in phase A */
  uint32_t n_union_dfas;  /* multi-pattern automata among n_dfas */
  uint32_t n_scan_streams; /* phase-A streams (value source x transformation chain) */
  uint32_t n_nfas;        /* @rx operators matched by NFA position tables (DFA over the state cap) */
  uint64_t source_digest;  /* FNV-1a 64 of the SecLang text + export list the ruleset was compiled from */
} gi_ruleset_info;

/* A byte range inside gi_batch.data. */
typedef struct {
  uint64_t off;
  uint32_t len;
  uint32_t _pad;
} gi_span;

/* One HTTP request: what ProcessConnection(client, cport, ...),
 * ProcessURI(uri, method, proto), AddRequestHeader(k, v) x hdr_count and
 * WriteRequestBody(body) receive. */
typedef struct {
  gi_span method;
  gi_span uri;
  gi_span proto;
  gi_span body;
  uint32_t hdr_begin; /* index into gi_batch.headers */
  uint32_t hdr_count;
  gi_span remote_addr;  /* ProcessConnection client address -> REMOTE_ADDR (may be empty) */
  uint32_t remote_port; /* -> REMOTE_PORT */
  uint32_t _pad;
  gi_span server_name;  /* Transaction.SetServerName -> SERVER_NAME (may be empty; coraza-proxy-wasm
                         * sets it from :authority without the port) */
} gi_request;

typedef struct {
  gi_span name;
  gi_span value;
} gi_header;

typedef struct {
  uint32_t n_req;
  const uint8_t* data; /* byte arena every gi_span points into */
  uint64_t data_len;
  const gi_request* reqs;
  const gi_header* headers;
  uint32_t n_headers;
} gi_batch;

/* Per-request verdict: coraza Interruption + matched-rule list + TX exports. */
typedef struct {
  int32_t rule_id;   /* interrupting rule id (0 = no interruption) */
  int32_t status;    /* Interruption.Status */
  uint8_t action;    /* GI_ACTION_* */
  uint8_t phase;     /* phase the interruption happened in */
  uint16_t flags;    /* GI_REQ_* */
  uint32_t match_cnt;                 /* matched rules (may exceed matched_cap) */
  int64_t tx_export[GI_MAX_EXPORTS];  /* Atoi of the exported TX values (0 if unset) */
  uint32_t capture_cnt;               /* capture records written (gi_results.captures) */
  uint32_t _pad;
} gi_verdict;

/* One observable capture (coraza rx.go FindStringSubmatch -> TX.<group>):
 * the top-level rule whose link captured, the group, and the captured bytes
 * at capture_bytes[row + off, + len).  Recorded for every capture whose
 * TX.0-TX.8 value a rule, macro or export can read (the compiler drops the
 * others: they change no output); in evaluation order. */
typedef struct {
  int32_t rule_id;
  uint32_t group;
  uint32_t off;
  uint32_t len;
} gi_capture;

typedef struct {
  gi_verdict* verdicts;   /* n_req entries */
  uint32_t* matched_ids;  /* n_req * matched_cap entries, row r = request r */
  uint32_t matched_cap;   /* must equal the ctx's matched_cap */
  /* optional (NULL: not fetched): n_req rows of capture_cap records and of
   * capture_bytes_cap bytes; the caps must equal the ctx's (gi_ctx_set_capture_cap) */
  gi_capture* captures;
  uint8_t* capture_bytes;
  uint32_t capture_cap;
  uint32_t capture_bytes_cap;
} gi_results;

/* Batch-level tallies (what bench/RCCL all-gathers across GPUs). */
typedef struct {
  uint64_t n_req;
  uint64_t n_interrupted;
  uint64_t n_matched_any;
  uint64_t n_error;
  uint64_t bytes_scanned; /* sum of raw request bytes (method+uri+proto+headers+body) */
  uint64_t matched_total;
  uint64_t n_pa_void;     /* requests whose phase-A arena overflowed (evaluated exhaustively) */
} gi_tally;

/* Detail tallies of the last batch (what the multi-GPU tally
 * all-gathers besides gi_tally): a histogram of the request's inbound anomaly
 * score -- the sum of the exported inbound_anomaly_score_pl1..pl4 values (what
 * CRS 949110 adds up; set even when a phase-2 attack rule interrupts before
 * 949061 sums blocking_inbound_anomaly_score), or the first exported TX value
 * when none of those is exported -- clamped to [0, GI_SCORE_BINS-1],
 * and per distinct rule id (ascending) the number of times it appears in the
 * matched-rule lists (MatchedRules) of the batch. */
#define GI_SCORE_BINS 64

typedef struct {
  uint64_t batches;
  double last_kernel_ms;   /* HIP-event time of the last inspection pipeline */
  double last_stage_ms;    /* H2D staging time of the last batch */
  uint64_t last_scratch_bytes;
  double last_collect_ms;  /* k_collect (ProcessURI / headers / cookies) */
  double last_scan_ms;     /* k_scan (phase A: automata over the transformed values) */
  double last_eval_ms;     /* k_eval (phase B: rule interpreter, body, verdicts) */
  double last_stream_ms;   /* k_stream (phase A: filters + transformation chains) */
  uint64_t last_pa_bytes;  /* phase-A arena bytes reserved for the batch */
  uint64_t diag[8];        /* diagnostic counters of the last batch (GI_DIAG=1) */
  uint32_t n_launches;     /* kernel launches of the last pipeline run */
  uint32_t _pad;
  double launch_ms[GI_STATS_LAUNCHES];    /* HIP-event time of each launch */
  uint64_t launch_alg_bytes[GI_STATS_LAUNCHES]; /* algorithmic bytes each launch must move */
  char launch_name[GI_STATS_LAUNCHES][16];
  uint64_t launch_steps[GI_STATS_LAUNCHES];     /* automaton byte-steps of each k_scan launch (secondary bound) */
  uint64_t gate_requests;  /* requests with a body the phase gate's first stage evaluated (0: no gate) */
  uint64_t gate_pending;   /* of which undecided there: scanned and evaluated again by the body stage */
} gi_stats;

/* ABI revision of the structs above (gi_batch, gi_results, gi_verdict,
 * gi_tally, gi_stats, ...).  It changes whenever one of them changes layout;
 * a binding checks gi_abi_version() == GI_ABI_VERSION before passing any of
 * them (INTEGRATION.md lists the revisions). */
#define GI_ABI_VERSION 6
uint32_t gi_abi_version(void);

/* ------------------------------------------------------------ compile */
int gi_compile(const char* seclang, size_t n, const gi_compile_opts* opts, gi_ruleset** out,
               char* err, size_t errcap);
void gi_ruleset_free(gi_ruleset* rs);
int gi_ruleset_info_get(const gi_ruleset* rs, gi_ruleset_info* out);
/* ids of the exported TX names, in order (for result decoding) */
int gi_ruleset_export_name(const gi_ruleset* rs, uint32_t i, char* buf, size_t cap);
/* GPU artifact of a compiled ruleset (the compile path's artifact
 * emitter): the whole compiled program as one versioned, checksummed blob,
 * served next to RuleSetEntry.Rules (internal/rulesets/cache/cache.go:32-36)
 * and keyed like it by the entry UUID (cache.go:81-100), so a data plane that
 * polls GET /rules/<key>/latest (server.go:163-181) loads the program instead
 * of recompiling the SecLang text.
 *   gi_ruleset_save  writes at most cap bytes; returns the artifact size (call
 *                    with cap 0 to size the buffer) or a negative GI_* code.
 *   gi_ruleset_load  GI_EINVAL + message for a truncated, corrupted,
 *                    other-version or other-compiler artifact, and for one
 *                    whose records index outside their tables (every index
 *                    and offset a kernel dereferences is bounds-checked: the
 *                    checksum is not authentication). */
int64_t gi_ruleset_save(const gi_ruleset* rs, uint8_t* buf, size_t cap);
int gi_ruleset_load(const uint8_t* buf, size_t n, gi_ruleset** out, char* err, size_t errcap);
/* Compiler revision string.  It is part of every source digest and artifact:
 * an artifact from another compiler revision fails gi_ruleset_load, and the
 * data plane recompiles RuleSetEntry.Rules instead. */
const char* gi_compiler_rev(void);

/* JSON description of the phase-A scan plan (streams, jobs, automata sizes).
 * Writes at most cap bytes (NUL-terminated); returns the full length
 * (excluding the NUL), or a negative GI_* code. */
int64_t gi_ruleset_describe(const gi_ruleset* rs, char* buf, size_t cap);

/* ------------------------------------------------------------ context */
int gi_ctx_create(const gi_ruleset* rs, int device, uint32_t matched_cap, gi_ctx** out);
/* Hot swap: the ctx evaluates rs from the next staged batch on (the data
 * plane's live reload when /latest reports a new UUID, server.go:163-181;
 * KATs reconcile_test.go:72-88).  Device buffers are reused; a staged batch
 * is dropped and must be staged again.  rs must outlive its use by the ctx. */
int gi_ctx_swap_ruleset(gi_ctx* ctx, const gi_ruleset* rs);
/* Capture-record capacity per request (default 8 records, 512 bytes); takes
 * effect from the next staged batch.  Overflow sets GI_REQ_CAPTURE_TRUNC. */
int gi_ctx_set_capture_cap(gi_ctx* ctx, uint32_t records, uint32_t bytes);
void gi_ctx_free(gi_ctx* ctx);
const char* gi_last_error(const gi_ctx* ctx);

/* One-shot: stage (H2D) + run + fetch (D2H), synchronous. */
int gi_inspect_batch(gi_ctx* ctx, const gi_batch* in, gi_results* out);

/* Split form used by the benchmark (HBM-resident timing):
 *   gi_stage_batch   copy the batch into device memory and lay out scratch
 *   gi_run_staged    run the inspection kernels on the staged batch
 *                    (asynchronous on the ctx stream)
 *   gi_sync          wait for the ctx stream
 *   gi_fetch_results copy verdicts / matched ids back */
int gi_stage_batch(gi_ctx* ctx, const gi_batch* in);
int gi_run_staged(gi_ctx* ctx);
int gi_sync(gi_ctx* ctx);
int gi_fetch_results(gi_ctx* ctx, gi_results* out);
int gi_tally_get(gi_ctx* ctx, gi_tally* out);
/* score_hist: GI_SCORE_BINS entries (may be NULL).  rule_ids / rule_hits:
 * cap entries each (may be NULL); *n_rules = the ruleset's distinct rule ids
 * (GI_ETRUNC when cap is smaller and the arrays are given).  With every
 * array NULL it only reports *n_rules (no batch needed). */
int gi_tally_detail_get(gi_ctx* ctx, uint64_t* score_hist, uint32_t* rule_ids, uint64_t* rule_hits, uint32_t cap,
                        uint32_t* n_rules);
int gi_stats_get(gi_ctx* ctx, gi_stats* out);
/* Opaque hipStream_t of the ctx (for HIP-event timing by the caller). */
void* gi_ctx_stream(gi_ctx* ctx);
/* Optional pinned-host fast path (input buffers are borrowed
 * per call, "with an optional pinned-host fast path"): page-lock a caller
 * buffer that later gi_batch arrays point into, so gi_stage_batch's H2D copies
 * run as DMA without a bounce buffer.  The caller keeps ownership; unregister
 * before freeing it.  GI_ENODEV / GI_ENOMEM when the HIP runtime refuses. */
int gi_host_register(gi_ctx* ctx, void* p, size_t n);
int gi_host_unregister(gi_ctx* ctx, void* p);

/* ---------------------------------------------------------- CPU baseline
 * with no Coraza Go toolchain on the GPU box, the reported CPU
 * number is "the build's own C++ CPU restatement, multi-threaded on all cores
 * and labelled as such (not Coraza)".  This is the engine's own per-request
 * interpreter (kernels.hip: ProcessURI / headers / cookies, body processors,
 * transformations, operators incl. libinjection, the rule walk) compiled a
 * second time for the host and run one request per thread at a time over
 * n_threads threads (0: all cores), without phase A: every rule link is
 * evaluated by the interpreter.  Results land in out->verdicts /
 * out->matched_ids (captures are not recorded).  *eval_seconds (optional) is
 * the wall time of the evaluation alone.  It is a baseline, never a fallback:
 * gi_inspect_* only run on the GPU. */
int gi_cpu_baseline_inspect(const gi_ruleset* rs, const gi_batch* in, gi_results* out, uint32_t n_threads,
                            double* eval_seconds);

/* ------------------------------------------------------- self-test hooks
 * Compiler self-tests only: run a host-built automaton on the host.  These
 * never take part in gi_inspect_* (which only runs on the GPU). */
int gi_selftest_regex(const char* pattern, size_t plen, const uint8_t* s, size_t n, uint32_t* n_states);
/* The same over n strings (data + offs[k] .. offs[k + 1]), one build:
 * out[k] = 1 on a match.  *n_states = 0 when the DFA exceeds the state cap
 * and the NFA tables (the compiler's fallback for @rx) answered. */
int gi_selftest_regex_many(const char* pattern, size_t plen, const uint8_t* data, const uint64_t* offs, uint32_t n,
                           uint8_t* out, uint32_t* n_states);
/* The capture submatch program (pike.h, the code k_eval runs) on the host:
 * "(?sm)" + pattern over s -> 1 on a match with caps[0 .. *nslot) = group
 * byte offsets (-1: not set), 0 without a match, or a negative GI_* code.
 * caps needs 18 entries. */
int gi_selftest_capture(const char* pattern, size_t plen, const uint8_t* s, size_t n, int32_t* caps,
                        uint32_t* nslot);
/* Host emulation of the phase-A scan over every job image of a compiled
 * ruleset (bounds + image walk vs the global tables).  0 = consistent. */
int gi_selftest_plan(const gi_ruleset* rs, char* err, size_t errcap);
/* The transformation identity-trigger table the kernels use (triggers[code],
 * code < n_codes) and the byte summary of every byte value (256 entries). */
int gi_selftest_triggers(uint32_t* triggers, uint32_t n_codes, uint32_t* byte_summaries);

#ifdef __cplusplus
}
#endif
#endif /* GPUINSPECT_H */
