// Kernel-side batch descriptor and launch entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuinspect.h"
#include "gi_program.h"

namespace gi {

struct Slot;  // TX variable (kernels.hip)

// Per-request scratch layout (computed by the host from request lengths when
// the batch is staged; see runtime.cpp gi_stage_batch).  Region =
// [256 B ReqHdr][cap_f fields][TX slots][cap_b bytes][2 x cap_t][2 x cap_mt].
struct ReqLayout {
  uint64_t base;   // byte offset of the request's region in DBatch.scratch
  uint32_t cap_f;  // field records
  uint32_t cap_b;  // decoded-bytes arena
  uint32_t cap_t;  // each of the two transformation buffers
  uint32_t cap_mt; // macro expansion scratch == TX string arena size
  uint64_t vmap_bit;   // first word of the request's value signatures in DBatch.vmap
  uint32_t vmap_bits;  // 2 x cap_f signatures: word 2f = value of field f, 2f + 1 = its key
  uint32_t hset_mask;  // exact phase-A hit set: capacity - 1 (a power of two minus one)
  uint64_t hset_word;  // its first word in DBatch.hset: [0] overflow flag, [1, cap] keys
  uint32_t dyn_cap;    // dynamic TX area (macro-key setvars): entries
  uint32_t dyn_capb;   // and bytes (0 / 0: the program has none)
  uint32_t mv_cap_e;   // MATCHED_VARS entries / arena bytes one rule can record (kernels.hip MvState;
  uint32_t mv_cap_a;   // 0 / 0: the program reads no matched-variable state)
  uint64_t cap_off;    // observable captures: the request's area in DBatch.cappool (chunk-relative)
};

struct DBatch {
  const uint8_t* data;
  const gi_request* reqs;
  const gi_header* headers;
  uint32_t n_req;
  uint32_t mcap;
  uint8_t* scratch;
  uint8_t* cappool;           // capture areas of the running chunk (CapHdr + pike workspace + group values)
  const DProgram* prog;       // the program in device memory (k_eval's interpreter reads it through this)
  const ReqLayout* layout;
  gi_verdict* verdicts;
  uint32_t* matched;
  uint32_t* caprec;           // [n_req][crcap] gi_capture records (4 words)
  uint8_t* capbytes;          // [n_req][cbcap] capture bytes
  uint32_t crcap, cbcap;
  unsigned long long* tally;  // gi_tally counters
  uint32_t* tally_ext;        // [GI_SCORE_BINS] score histogram, then per distinct rule id match counts
  uint32_t* hits;             // phase-A hit words [ceil(n_hit_slots/32)][n_req]
  uint32_t* vmap;             // phase-A value map: per scanned (field, side) a u32 signature, bit (slot % 32)
                              // of every hit slot the value set (k_eval re-tests a link only on values with its bit)
  uint32_t* hset;             // exact phase-A hit sets: per request an open-addressing table of
                              // (slot, value index, maybe) keys (kernels.hip hset_key)
  const uint32_t* body_list;  // requests with a body, longest first (k_body: one wave each)
  uint32_t n_body;
  uint32_t n_mp_body;         // of which multipart (k_mpparse)
  Slot* txslots;       // TX variables [n_slots][n_req] (k_eval)
  // phase A (see kernels.hip "phase A")
  uint32_t* bcounts;          // [k_collect blocks][GI_NCLS] item counts per length class
  uint32_t* boffs;            // [k_collect blocks][GI_NCLS] item offsets within the class
  uint32_t* ctot;             // [GI_NCLS] items per class (k_ioffsets)
  uint32_t* cbase;            // [GI_NCLS] first item of each class (k_ibases)
  uint32_t* ibk;              // [GI_NB] (base, count), [GI_NB] item-wave base, total item waves
  void* items;                // Item[items_cap]
  uint64_t* igm;              // [items_cap] global filters admitting each item (k_stream -> k_scan)
  uint8_t* lscratch;          // per-lane HBM transformation buffers (2 x lcap per k_stream lane)
  uint32_t lcap;
  uint32_t* pool;             // queue-block words
  uint64_t pool_cap;          // words
  unsigned long long* pool_used;
  uint2* qblk;                // [stream][qcap] queue blocks {word offset, nv | nw << 8}
  unsigned long long* acct;   // algorithmic-byte counters: [0..5) item bytes per bucket, [5..10) queue
                              // words written per k_stream bucket, [10..13) queue words read per k_scan launch,
                              // [13..16) automaton byte steps per k_scan launch
  unsigned long long* acct3;  // [0..5) items per length bucket, summed over the chunks of a run
  unsigned long long* acct2;  // byte steps: [0..5) value bytes into stream chains per k_stream bucket,
                              // [5] value bytes through libinjection (k_detect)
  uint32_t qcap;
  void* slow;                 // SlowEnt[slow_cap]
  uint32_t* slow_count;
  uint32_t slow_cap;
  uint8_t* slow_bytes;
  uint64_t slow_bytes_cap;
  unsigned long long* slow_used;
  uint2* long_list;           // (item, stream) of long values (k_stream -> k_long, one wave each)
  uint32_t* long_count;
  uint32_t long_cap;
  uint32_t long_grid;         // k_long workgroups (each owns two long_bufcap buffers)
  uint8_t* long_buf;
  uint64_t long_bufcap;
  void* det;                  // DetEnt[det_cap]: @detectSQLi/@detectXSS candidates (k_stream -> k_detect)
  uint32_t* det_count;
  uint32_t det_cap;
  uint8_t* det_bytes;
  uint64_t det_bytes_cap;
  unsigned long long* det_used;
  unsigned long long* diag;   // optional diagnostic counters (gi_stats.diag)
  unsigned long long* vcause; // [6] phase-A void events per cause (GI_VOID_*, kernels.hip)
  uint32_t* dbg;              // debug-build bounds-violation record (-DGI_DEBUG)
  unsigned long long* prof;   // GI_PROF=1: k_eval cycle / rule counters (stderr at gi_sync)
  uint64_t items_cap;
  uint32_t n_hit_slots;
  uint32_t* wlist;            // requests k_eval hands to k_eval_wave (a wave each)
  uint32_t* wcount;
  uint32_t wave_fields;       // k_eval_wave: requests with this many fields (0: none)
  uint32_t wave_rules;        // k_eval_wave: every request when the program walks this many rules (0: never)
  uint32_t mp_wave;            // k_mpparse: parts split over the lanes (wave_multipart; GI_MP_WAVE=0: lane 0 alone)
  uint32_t bparse_wave;        // k_bparse: JSON bodies parsed by the whole wave (wave_parse_json; GI_BPARSE_WAVE=0: lane 0)
  uint32_t bparse_lds;        // k_bparse: JSON bodies up to this many bytes are parsed from LDS (its dynamic LDS)
  uint32_t rstride;           // request stride of the request-major SoA arrays (hits, txslots): the staged
                              // batch's size (a chunk view of it has n_req <= rstride)
  // Phase-1 gate (launch_pipeline): stage 1 runs phase A over the phase-1
  // fields and evaluates phase 1 (whole requests without a body); a request a
  // phase-1 rule interrupted is final there -- coraza never calls
  // WriteRequestBody for it.  Stage 2 parses the bodies of the other (pending)
  // requests, runs phase A over their body fields and evaluates them in full.
  uint32_t stage;             // 0: one pass (no gate); 1: phase-1 stage; 2: body stage
  uint32_t gate;              // the host allows the gate (GI_GATE=0 turns it off)
  uint8_t* pend;              // [n_req] stage 1 -> 2: 1 = the request continues to the body stage
  uint32_t* plist;            // the pending requests (stage-1 k_eval appends), *pcount of them
  uint32_t* eorder;           // k_eval's request order (nullptr: identity): requests grouped by their count of
                              // set phase-A hit bits, so a wave's lanes walk similar rule paths (k_eord_*)
  uint32_t* eord_bins;        // [GI_EORD_BINS] counts, then [GI_EORD_BINS] cursors (ctr)
  uint8_t* eord_key;          // per request: its bin (k_eord_count -> k_eord_scatter)
  // header dedup (k_collect -> k_dspread): keys (hash | 1, 0 = empty) and per entry
  // (canonical request + 1) << 32 | (field * 2 + side), 0 until published; nullptr: off
  unsigned long long* hdkeys;
  unsigned long long* hdinfo;
  uint32_t* hdref;            // [2 * header slot + side]: a copy's canonical entry + 1 (0: none)
  uint32_t hdmask;
  uint32_t* pcount;
  uint32_t wave_stage2;       // the body stage's pending requests all go to k_eval_wave (GI_EVAL_WAVE_STAGE2=0: by size)
  uint32_t body_tiles;        // k_body runs its chunkable transformations LDS-tiled (GI_BODY_TILES=0: off)
  // k_detect's memo of libinjection results by value (kernels.hip det_memo):
  // the same header / cookie value recurs across requests (User-Agent,
  // Referer); open addressing on a 64-bit hash, entries verified byte for byte
  unsigned long long* dmemo_keys;  // [dmemo_mask + 1] (0: empty); nullptr: no memo
  uint4* dmemo_info;               // per entry: canonical copy offset (lo, hi) in det_bytes, length, state bits
  uint32_t dmemo_mask;
  uint32_t dmemo_min;  // shortest value the memo serves (GI_DET_MEMO_MIN; shorter ones are cheaper to detect)
};

// k_scan launch plan: job lists for the small-LDS and big-LDS launches.
struct ScanLaunch {
  const uint32_t* jobs[2];  // device job-index lists
  uint32_t n_jobs[2];
  uint32_t lds[2];          // dynamic LDS bytes per workgroup
  uint32_t blocks[3];       // resident workgroups (persistent grid); [2] = HBM-image launch
  uint32_t rpl[2];          // requests per lane per unit
  const uint32_t* global_jobs;  // jobs whose image is read from HBM (too large for LDS)
  uint32_t n_global;
  uint32_t mode;                // debugging switches (GI_SCAN_MODE), 0 in production
};

#define GI_SLOT_BYTES 16      // sizeof(Slot) (kernels.hip): a TX variable of one request
#define GI_NCLS 2320          // item classes: 16 source groups x length classes (kernels.hip item_class)
#define GI_RHIST_LDS 1024     // per-rule match counts k_eval aggregates in LDS (more rules: global atomics)
#define GI_STREAM_GRID 8192  // k_stream workgroups (64 lanes) per bucket launch (~8 waves/SIMD)
#define GI_PCHUNK 2048       // pool words a k_stream wave reserves at a time
#define GI_LONG_MIN 2048     // items at least this long take k_long (one wave per (item, stream)), not the queue
#define GI_LONG_GRID 512     // k_long workgroups (at most)
#define GI_LONG_BUDGET (4ull << 30)  // bytes of k_long chain buffers (runtime.cpp gi_stage_batch)
#define GI_EVAL_LDS_WORDS 16          // k_eval keeps a request's hit words in LDS up to this many
#define GI_EVAL_WAVE_LDS_WORDS 4096  // k_eval_wave keeps a request's hit words in LDS up to this many
#define GI_EVAL_WAVE_FIELDS 4096     // default k_eval_wave thresholds (GI_EVAL_WAVE_FIELDS / _RULES env)
#define GI_EVAL_WAVE_RULES 2048
#define GI_BPARSE_LDS 0              // k_bparse LDS copy of JSON bodies up to this size (GI_BPARSE_LDS env; 0: off --
                                     // measured: 32 KB made C3's k_bparse 81 -> 272 ms, the LDS cut its occupancy)
#define GI_BPARSE_WIN 4096           // wave_parse_json's LDS window over a JSON body (GI_BPARSE_WIN env, >= 2048)
#define GI_EORD_BINS 32               // k_eval order: bins of hit-bit counts
#define GI_EORD_GRID 512              // k_eord_* workgroups (each a contiguous chunk of requests)
#define GI_GATE_PENDING_MAX 0.5       // the adaptive gate runs while at most this share of body requests stays pending
#define GI_CHUNK_POOL_WORDS 16e9     // queue-pool words (estimate) one request chunk of a batch may need

// Resident k_scan workgroups (1024 threads) with lds_bytes of dynamic LDS.
uint32_t scan_resident_blocks(uint32_t lds_bytes);
// Raise the dynamic-LDS limit of k_scan for images above 64 KiB.
void scan_allow_lds(uint32_t lds_bytes);

// k_collect -> k_stream -> k_scan (small, big) -> k_eval on `stream`;
// ev (optional) = 3 events recorded after k_collect, k_stream and k_scan.
// Per-launch HIP events of one pipeline run (ev[0] before the first launch,
// ev[k + 1] after launch k).
#define GI_MAX_LAUNCHES 256  // launches of one run (a chunked batch repeats the pipeline; gi_stats sums by name)
struct LaunchLog {
  hipEvent_t ev[GI_MAX_LAUNCHES + 1];
  const char* name[GI_MAX_LAUNCHES];
  int n;
};

// stop_after > 0 (debugging): launch only the first stop_after kernels and
// synchronise after each, printing the first failing one.
// tally_ids: the ruleset's distinct rule ids, ascending (k_tally bins).
// CPU baseline: request 0 of B through the interpreter compiled for the host (kernels.hip)
void cpu_inspect_one(const DProgram& P, const DBatch& B);
void launch_pipeline(const DProgram& P, const DBatch& B, const ScanLaunch& S, hipStream_t stream, hipEvent_t* ev,
                     int stop_after, LaunchLog* log, const uint32_t* tally_ids, uint32_t n_tally_ids);

}  // namespace gi
