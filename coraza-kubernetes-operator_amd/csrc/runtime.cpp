// Host runtime of the C ABI (include/gpuinspect.h): compile, device context,
// batch staging (H2D + per-request scratch layout), launch, result fetch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/gpuinspect.h"
#include "artifact.h"
#include "compile.h"
#include "gi_kernels.h"
#include "unicode_tables.h"

using namespace gi;

struct gi_ruleset {
  Program prog;
  gi_ruleset_info info;
};

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <class T>
hipError_t upload(DevBuf* b, const std::vector<T>& v, hipStream_t s) {
  size_t n = std::max<size_t>(v.size() * sizeof(T), 16);
  hipError_t e = b->ensure(n);
  if (e != hipSuccess) return e;
  if (!v.empty()) e = hipMemcpyAsync(b->p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  return e;
}

const std::vector<std::string> kDefaultExports = {
    "blocking_inbound_anomaly_score", "inbound_anomaly_score_pl1", "inbound_anomaly_score_pl2",
    "inbound_anomaly_score_pl3", "inbound_anomaly_score_pl4", "detection_inbound_anomaly_score",
    "anomaly_score"};

// Phase-A arena sizing factor (GI_PA_FACTOR overrides; see gi_stage_batch).
// Queue-pool sizing factor (GI_POOL_FACTOR overrides; see gi_stage_batch).
double pool_factor_env() {
  const char* v = getenv("GI_POOL_FACTOR");
  double f = v ? atof(v) : 0.0;
  return f > 0 ? f : 1.0;
}

}  // namespace

struct gi_ctx {
  const gi_ruleset* rs = nullptr;
  int device = 0;
  uint32_t mcap = 64;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;
  DProgram prog{};
  std::vector<DevBuf> pbufs;
  // batch buffers
  DevBuf cappool;  // capture areas of one request chunk (reused by every chunk)
  DevBuf progdev;  // the DProgram struct itself in device memory (DBatch.prog)
  DevBuf data, reqs, hdrs, layout, scratch, verdicts, matched, tally, tally_ext, hits, vmap, hset, blist, joblist, txslots;
  DevBuf tally_idbuf;                  // distinct rule ids, ascending (k_tally bins)
  DevBuf caprec, capbytes;             // capture records / bytes (observable captures)
  uint32_t crcap = 8, cbcap = 512;     // per request (gi_ctx_set_capture_cap)
  uint32_t staged_crcap = 8, staged_cbcap = 512;
  bool cap_on = false;
  std::vector<uint32_t> tally_ids;
  // phase A
  DevBuf bcounts, boffs, items, igm, lscratch, pool, qblk, ctr, slow, slow_bytes, det, det_bytes, long_list, long_buf, wlist;
  DevBuf pend, plist;  // phase-1 gate (launch_pipeline): pending flags + list
  DevBuf eorder, ekey;  // k_eval's request order (k_eord_*: requests grouped by phase-A hit count), bins
  DevBuf hdkeys, hdinfo, hdref;  // header dedup table (k_collect / k_dspread), copies' entries
  uint32_t hdmask = 0;
  DevBuf dmemo_keys, dmemo_info;  // k_detect's detector-result memo
  uint32_t dmemo_mask = 0;
  uint32_t long_cap = 0, long_grid = GI_LONG_GRID;
  uint32_t wave_fields = GI_EVAL_WAVE_FIELDS, wave_rules = GI_EVAL_WAVE_RULES;  // k_eval_wave thresholds
  // The phase gate (kernels.hip launch_pipeline) pays off when its first stage
  // decides many of the requests with a body; when most stay pending (the body
  // stage scans and evaluates them anyway) it costs a second evaluation.  The
  // context tracks the pending share of its gated batches and runs ungated
  // while it stays above GI_GATE_PENDING_MAX, re-probing every 16th batch.
  // Results do not depend on the choice (both forms are exact).
  double gate_pending_share = -1.0;  // last gated batch (-1: none yet)
  bool gate_ran = false;             // the batch in flight ran gated
  // A staged batch runs as consecutive request chunks, each a full pipeline
  // pass over its requests, so the phase-A buffers (items, queue pool, detect
  // / slow / long lists) are sized for one chunk, not for the whole batch.
  struct Chunk {
    uint32_t r0, n;          // requests [r0, r0 + n)
    uint32_t blist_off;      // its body list (longest first) in blist
    uint32_t n_body, n_mp;
  };
  std::vector<Chunk> chunks;
  double chunk_pool_words = GI_CHUNK_POOL_WORDS;
  // capture pool a chunk may use (GI_CHUNK_CAP_BYTES env): C2's 1M requests need
  // ~8 GB (one chunk); a ruleset with a huge capture regex runs in more chunks
  uint64_t chunk_cap_bytes = 16ull << 30;
  ReqLayout* lay_host = nullptr;  // page-locked host copy of the staged layout
  uint32_t lay_host_cap = 0;
  bool stage_prof = false;
  uint32_t bparse_lds = GI_BPARSE_LDS;  // GI_BPARSE_LDS env
  uint32_t bparse_wave = 1;              // GI_BPARSE_WAVE env (0: JSON bodies on lane 0, A/B)
  uint32_t bparse_win = GI_BPARSE_WIN;   // GI_BPARSE_WIN env: wave_parse_json's LDS window
  uint64_t max_body = 0;                // longest body of the staged batch        // GI_STAGE_PROF=1: gi_stage_batch phase times on stderr  // queue-pool estimate a chunk may reach (GI_CHUNK_POOL_WORDS env)
  uint64_t long_bufcap = 0;
  uint32_t lcap = 0, qcap = 0, slow_cap = 0, det_cap = 0;
  uint64_t pool_cap = 0, slow_bytes_cap = 0, items_cap = 0, det_bytes_cap = 0;
  bool diag_on = false, prof_on = false;
  DevBuf prof;
  int stop_after = 0;  // debugging: launch only the first N pipeline kernels, synchronising after each
  ScanLaunch scan{};
  uint32_t hit_words = 0;
  uint64_t vmap_words = 0;  // value map (DBatch.vmap)
  uint64_t hset_words = 0;  // exact hit sets (DBatch.hset)
  uint32_t n_body = 0;      // requests with a body (DBatch.body_list)
  uint32_t n_mp_body = 0;   // of which multipart
  hipEvent_t evs[3] = {nullptr, nullptr, nullptr};
  LaunchLog log{};
  uint64_t raw_nobody = 0, raw_all = 0;  // batch bytes (algorithmic-byte accounting)
  uint32_t n_req = 0;
  bool staged = false, ran = false;
  gi_stats stats{};
};

static int fail(gi_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}
static int hip_fail(gi_ctx* c, hipError_t e, const char* what) {
  return fail(c, e == hipErrorOutOfMemory ? GI_ENOMEM : GI_ENODEV,
              std::string(what) + ": " + hipGetErrorString(e));
}

extern "C" {

static void fill_info(gi_ruleset* rs) {
  const Program& P = rs->prog;
  rs->info.n_rules = (uint32_t)P.top.size();
  rs->info.n_links = (uint32_t)P.rules.size();
  rs->info.n_dfas = (uint32_t)P.dfas.size();
  rs->info.n_tx_slots = P.n_slots;
  rs->info.n_scan_jobs = (uint32_t)P.jobs.size();
  rs->info.n_scan_streams = (uint32_t)P.streams.size();
  rs->info.n_hit_slots = P.n_hit_slots;
  rs->info.n_union_dfas = P.n_union_dfas;
  rs->info.n_nfas = (uint32_t)P.nfas.size();
  rs->info.program_bytes = P.rules.size() * sizeof(DRule) + P.vars.size() * sizeof(DVarRef) +
                           P.ops.size() * sizeof(DOp) + P.acts.size() * sizeof(DAction) +
                           P.trans.size() * 2 + P.u8pool.size() + P.nranges.size() * 4 + P.strpool.size() +
                           P.dfas.size() * sizeof(DDfa) + P.tparts.size() * sizeof(DTmplPart) +
                           P.u64pool.size() * 8 + P.streams.size() * sizeof(DStream) +
                           P.filters.size() * sizeof(DFilter) + P.jobs.size() * sizeof(DJob) +
                           P.jdfas.size() * sizeof(DJobDfa) + P.pats.size() * sizeof(DPat) +
                           P.svals.size() * sizeof(DScanVal) + P.images.size();
  rs->info.source_digest = P.source_digest;
  if (getenv("GI_PLAN")) {  // diagnostics: the phase-A plan (streams -> jobs -> images)
    for (const DRule& R : P.rules)
      if (R.op >= 0 && P.ops[R.op].nfa >= 0) {
        const DNfa& N = P.nfas[P.ops[R.op].nfa];
        fprintf(stderr, "rule %d: NFA tables %d (dfa %d) pos %u words %u classes %u nr %u\n", R.id, P.ops[R.op].nfa,
                P.ops[R.op].dfa, N.n_pos, N.words, N.n_classes, N.nr_cnt);
      }
    for (size_t k = 0; k < P.streams.size(); k++) {
      const DStream& S = P.streams[k];
      fprintf(stderr, "stream %zu chain", k);
      for (uint32_t q = 0; q < S.tchain_len; q++) fprintf(stderr, " %u", (unsigned)P.tchains[S.tchain_off + q]);
      fprintf(stderr, " | filters %u vals %u kinds %x:", S.filt_count, S.val_count, S.kind_mask);
      for (uint32_t j = S.job_begin; j < S.job_begin + S.job_count; j++)
        fprintf(stderr, " job%u(%u dfa, %u B%s%s)", j, P.jobs[j].jdfa_count, P.jobs[j].img_bytes, P.jobs[j].lds ? "" : " hbm",
                P.jobs[j].big ? " big" : "");
      fprintf(stderr, "\n");
    }
  }
}

int gi_compile(const char* seclang, size_t n, const gi_compile_opts* opts, gi_ruleset** out, char* err,
               size_t errcap) {
  if (!seclang || !out) return GI_EINVAL;
  *out = nullptr;
  std::vector<std::string> exports;
  if (opts && opts->tx_exports) {
    for (const char* const* p = opts->tx_exports; *p; p++) exports.push_back(*p);
  } else {
    exports = kDefaultExports;
  }
  if (exports.size() > GI_MAX_EXPORTS) exports.resize(GI_MAX_EXPORTS);
  auto* rs = new gi_ruleset();
  std::string msg;
  std::string digest_input(seclang, n);
  for (const auto& x : exports) digest_input.append("\0export:", 8).append(x);
  digest_input.append("\0compiler:", 10).append(kCompilerRev);
  std::map<std::string, std::string> data_files;
  if (opts && opts->n_data_files) {
    if (!opts->data_file_names || !opts->data_file_data || !opts->data_file_lens) {
      delete rs;
      return GI_EINVAL;
    }
    for (uint32_t i = 0; i < opts->n_data_files; i++) {
      if (!opts->data_file_names[i] || (!opts->data_file_data[i] && opts->data_file_lens[i])) {
        delete rs;
        return GI_EINVAL;
      }
      std::string body(opts->data_file_data[i] ? opts->data_file_data[i] : "", opts->data_file_lens[i]);
      digest_input.append("\0file:", 6).append(opts->data_file_names[i]).append("\0", 1).append(body);
      data_files[opts->data_file_names[i]] = std::move(body);
    }
  }
  int rc = compile_program(std::string(seclang, n), exports, opts ? opts->dfa_state_cap : 0, &rs->prog, &msg,
                           &data_files);
  if (rc != 0) {
    if (err && errcap) {
      size_t k = std::min(errcap - 1, msg.size());
      memcpy(err, msg.data(), k);
      err[k] = 0;
    }
    delete rs;
    return rc == -1 ? GI_EPARSE : GI_EUNSUPPORTED;
  }
  rs->prog.source_digest = gi::fnv64((const uint8_t*)digest_input.data(), digest_input.size());
  fill_info(rs);
  *out = rs;
  return GI_OK;
}

int64_t gi_ruleset_save(const gi_ruleset* rs, uint8_t* buf, size_t cap) {
  if (!rs) return GI_EINVAL;
  const std::vector<uint8_t> a = gi::serialize_program(rs->prog);
  if (buf && cap) memcpy(buf, a.data(), std::min(cap, a.size()));
  return (int64_t)a.size();
}

int gi_ruleset_load(const uint8_t* buf, size_t n, gi_ruleset** out, char* err, size_t errcap) {
  if (!buf || !out) return GI_EINVAL;
  *out = nullptr;
  auto* rs = new gi_ruleset();
  std::string msg;
  if (!gi::deserialize_program(buf, n, &rs->prog, &msg)) {
    if (err && errcap) {
      size_t k = std::min(errcap - 1, msg.size());
      memcpy(err, msg.data(), k);
      err[k] = 0;
    }
    delete rs;
    return GI_EINVAL;
  }
  fill_info(rs);
  *out = rs;
  return GI_OK;
}

void gi_ruleset_free(gi_ruleset* rs) { delete rs; }

const char* gi_compiler_rev(void) { return kCompilerRev; }
uint32_t gi_abi_version(void) { return GI_ABI_VERSION; }

int gi_ruleset_info_get(const gi_ruleset* rs, gi_ruleset_info* out) {
  if (!rs || !out) return GI_EINVAL;
  *out = rs->info;
  return GI_OK;
}

int gi_ruleset_export_name(const gi_ruleset* rs, uint32_t i, char* buf, size_t cap) {
  if (!rs || !buf || cap == 0) return GI_EINVAL;
  if (i >= rs->prog.export_names.size()) return GI_EINVAL;
  const std::string& s = rs->prog.export_names[i];
  size_t k = std::min(cap - 1, s.size());
  memcpy(buf, s.data(), k);
  buf[k] = 0;
  return GI_OK;
}

int64_t gi_ruleset_describe(const gi_ruleset* rs, char* buf, size_t cap) {
  if (!rs) return GI_EINVAL;
  const std::string& s = rs->prog.plan_json;
  if (buf && cap) {
    size_t k = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return (int64_t)s.size();
}

// Uploads (or replaces) the context's device copy of a compiled ruleset.
// The new program is validated and uploaded into fresh buffers first; the
// context switches to it (and frees the old buffers) only once every step
// succeeded, so a failed swap leaves the old ruleset fully in place.  The
// staged batch is dropped (its scratch layout depends on the program).
// Every DProgram field from the compiled Program.  put(p, bytes) stores one
// table where the interpreter reads it and returns that address: HBM for a
// context (load_program), host memory for the CPU baseline
// (gi_cpu_baseline_inspect).  Returns nullptr or an error message.
}  // extern "C"
template <class Put>
static const char* fill_dprogram(const Program& P, DProgram& np, Put&& put, std::vector<uint32_t>& top_ph,
                                 uint32_t& n_ph1) {
  std::vector<uint32_t> lower;
  lower.reserve(GI_N_LOWER_PAIRS * 2);
  for (int i = 0; i < GI_N_LOWER_PAIRS; i++) {
    lower.push_back(kLowerPairs[i][0]);
    lower.push_back(kLowerPairs[i][1]);
  }
#define UP(field, vec, T) np.field = (const T*)put((vec).data(), (vec).size() * sizeof((vec)[0]));
  UP(rules, P.rules, DRule)
  // per-phase rule walks: rules of that phase plus phase-0 records (SecMarker),
  // in file order -- what RuleGroup.Eval(phase) visits
  top_ph.clear();
  n_ph1 = 0;
  for (int ph = 1; ph <= 2; ph++) {
    for (uint32_t ri : P.top)
      if (P.rules[ri].phase == 0 || P.rules[ri].phase == ph) top_ph.push_back(ri);
    if (ph == 1) n_ph1 = (uint32_t)top_ph.size();
  }
  UP(top, top_ph, uint32_t)
  // skipAfter jumps: for a walk entry whose rule has skipAfter, the position of
  // the first later entry of the same walk with that marker (or the walk's end)
  std::vector<uint32_t> top_jump(top_ph.size(), 0);
  for (size_t a = 0; a < top_ph.size(); a++) {
    const size_t end = a < n_ph1 ? n_ph1 : top_ph.size();
    const int32_t m = P.rules[top_ph[a]].skip_after;
    size_t j = a + 1;
    while (m >= 0 && j < end && P.rules[top_ph[j]].marker != m) j++;
    top_jump[a] = (uint32_t)(m >= 0 ? j : a + 1);
  }
  UP(top_jump, top_jump, uint32_t)
  UP(vars, P.vars, DVarRef)
  UP(excs, P.excs, DExc)
  UP(ops, P.ops, DOp)
  UP(acts, P.acts, DAction)
  UP(tparts, P.tparts, DTmplPart)
  UP(tmpls, P.tmpls, DTmpl)
  UP(tchains, P.tchains, uint8_t)
  UP(dfas, P.dfas, DDfa)
  UP(nfas, P.nfas, DNfa)
  UP(trans, P.trans, uint16_t)
  UP(u8pool, P.u8pool, uint8_t)
  UP(nranges, P.nranges, uint32_t)
  UP(strpool, P.strpool, uint8_t)
  UP(lower_pairs, lower, uint32_t)
  UP(slot_names, P.slot_names, uint32_t)
  UP(u64pool, P.u64pool, uint64_t)
  UP(streams, P.streams, DStream)
  UP(filters, P.filters, DFilter)
  UP(jobs, P.jobs, DJob)
  UP(jdfas, P.jdfas, DJobDfa)
  UP(images, P.images, uint8_t)
  UP(pats, P.pats, DPat)
  UP(svals, P.svals, DScanVal)
  std::vector<uint32_t> sfilt32(P.sfilt.begin(), P.sfilt.end());
  std::vector<uint32_t> tch32(P.tchains.begin(), P.tchains.end());
  UP(sfilt, sfilt32, uint32_t)
  UP(tchains32, tch32, uint32_t)
  UP(always_slots, P.always_slots, uint32_t)
  UP(body_links, P.body_links, uint32_t)
  UP(pikes, P.pikes, DPike)
  UP(pike_insts, P.pike_insts, DPikeInst)
  UP(pike_ranges, P.pike_ranges, uint32_t)
  // static TX slot by (lowercase) name, for keys a macro-key setvar expands to
  // at run time: open addressing on gi_fnv1a, entry = slot + 1 (0 empty)
  std::vector<uint32_t> shash;
  {
    uint32_t cap = 16;
    while (cap < 2 * P.n_slots) cap <<= 1;
    shash.assign(cap, 0);
    for (uint32_t sl = 0; sl < P.n_slots; sl++) {
      const uint32_t h = gi_fnv1a(&P.strpool[P.slot_names[2 * sl]], P.slot_names[2 * sl + 1], false);
      uint32_t i = h & (cap - 1);
      while (shash[i]) i = (i + 1) & (cap - 1);
      shash[i] = sl + 1;
    }
    np.slot_hash_mask = cap - 1;
  }
  UP(slot_hash, shash, uint32_t)
  UP(txrx, P.txrx, uint32_t)
  // folded TX snapshot as device Slot records (kernels.hip Slot: num | string
  // pointer into the device string pool, n, state)
  struct SnapDev {
    uint64_t v;
    uint32_t n, state;
  };
  static_assert(sizeof(SnapDev) == GI_SLOT_BYTES, "Slot layout");
  std::vector<SnapDev> snap(std::max<size_t>(P.tx_snap.size(), 1), SnapDev{0, 0, 0});
  for (size_t i = 0; i < P.tx_snap.size(); i++) {
    const DSnapSlot& z = P.tx_snap[i];
    snap[i].state = z.state;
    snap[i].n = z.state == 2 ? z.len : 0u;
    snap[i].v = z.state == 1 ? (uint64_t)z.num : z.state == 2 ? (uint64_t)(uintptr_t)(np.strpool + z.off) : 0ull;
  }
  UP(tx_snap, snap, uint8_t)
  UP(fold_ids, P.fold_ids, uint32_t)
  UP(fold_runs, P.fold_runs, uint32_t)
  UP(rule_groups, P.rule_groups, uint32_t)
#undef UP
  np.n_rm_groups = P.n_rm_groups;
  np.args_limit = P.args_limit;
  np.n_lower_pairs = GI_N_LOWER_PAIRS;
  // observable captures: per-request submatch workspace (kernels.hip CapHdr +
  // pike_match) and the TX slots of the keys "0".."8"
  np.cap_ws_words = 0;
  np.cap_groups = 0;
  for (const DPike& k : P.pikes) {
    // (a whole-value capture, (?sm)^.*$, runs no VM: the CapHdr alone)
    np.cap_ws_words = (uint32_t)std::max<uint64_t>(np.cap_ws_words, 16 + (k.whole ? 0 : pike_ws_words(k.n_inst, k.nslot)));
    np.cap_groups = std::max<uint32_t>(np.cap_groups, k.nslot / 2);
  }
  for (int g = 0; g < 9; g++) {
    np.cap_slots[g] = -1;
    for (uint32_t sl = 0; sl < P.n_slots && !P.pikes.empty(); sl++)
      if (P.slot_names[2 * sl + 1] == 1 && P.strpool[P.slot_names[2 * sl]] == (uint8_t)('0' + g)) np.cap_slots[g] = (int32_t)sl;
  }
  np.n_top = (uint32_t)P.top.size();
  np.top_begin[0] = 0;
  np.top_end[0] = n_ph1;
  np.top_begin[1] = n_ph1;
  np.top_end[1] = (uint32_t)top_ph.size();
  np.n_slots = P.n_slots;
  np.n_dyn_sites = (uint32_t)P.dyn_sites.size();
  if (P.tx_snap.size() != P.n_slots) return "folded TX snapshot size";
  // a folded run starts and ends inside the phase-1 walk, at its own rule
  for (uint32_t a = 0; a < n_ph1; a++) {
    const DRule& R = P.rules[top_ph[a]];
    if (!(R.flags & RF_FOLDED)) continue;
    if (4ull * R._pad2 + 3 >= P.fold_runs.size() || P.fold_runs[4 * R._pad2 + 2] <= a ||
        P.fold_runs[4 * R._pad2 + 2] > n_ph1)
      return "folded run out of range";
  }
  for (size_t a = n_ph1; a < top_ph.size(); a++)
    if (P.rules[top_ph[a]].flags & RF_FOLDED) return "folded rule outside phase 1";
  np.fold_on = P.fold_on;
  np.fold_nids = P.fold_nids;
  np.n_markers = P.n_markers;
  np.n_exports = (uint32_t)P.exports.size();
  // score histogram (k_tally): the sum of the exported inbound_anomaly_score_pl1..pl4 -- what
  // 949110 adds up, and, unlike the blocking score, set under a deny default (a phase-2
  // attack rule interrupts before 949061 sums it) -- else the first export
  np.hist_mask = 0;
  for (uint32_t i = 0; i < np.n_exports && i < 8; i++) {
    const std::string& nm = P.export_names[i];
    if (nm.size() == 25 && nm.compare(0, 24, "inbound_anomaly_score_pl") == 0 && nm[24] >= '1' && nm[24] <= '4')
      np.hist_mask |= 1u << i;
  }
  if (!np.hist_mask) np.hist_mask = 1;
  for (int i = 0; i < 8; i++) np.exports[i] = i < (int)P.exports.size() ? P.exports[i] : -1;
  np.rule_engine = P.rule_engine;
  np.body_access = P.body_access;
  np.mv_used = P.mv_used;
  np.body_partial = P.body_partial;
  np.body_limit = P.body_limit;
  np.n_det_streams = 0;
  for (uint32_t k = 0; k < (uint32_t)P.streams.size(); k++)
    if (P.streams[k].det_id != 0xFF && P.streams[k].det_id < GI_MAX_DET_STREAMS) {
      np.det_streams[P.streams[k].det_id] = k;
      np.n_det_streams = std::max(np.n_det_streams, (uint32_t)P.streams[k].det_id + 1);
    }
  np.n_jobs = (uint32_t)P.jobs.size();
  np.max_img_bytes = P.max_img_bytes;
  np.max_big_img_bytes = P.max_big_img_bytes;
  np.n_streams = (uint32_t)P.streams.size();
  np.n_always = (uint32_t)P.always_slots.size();
  np.n_body_links = (uint32_t)P.body_links.size();
  np.n_gfilters = (uint32_t)P.filters.size();
  np.item_singles = P.item_singles;
  for (int k = 0; k < 8; k++) np.item_sides[k] = P.item_sides[k];
  np.n_hit_slots = P.n_hit_slots;
  return nullptr;
}
extern "C" {

static int load_program(gi_ctx* c, const gi_ruleset* rs) {
  hipError_t e = hipSuccess;
  const Program& P = rs->prog;
  if (P.streams.size() > GI_MAX_STREAMS) return fail(c, GI_EINVAL, "ruleset has more phase-A streams than supported");
  std::vector<DevBuf> nbufs(48);
  DevBuf njoblist;
  DProgram np{};
  ScanLaunch nscan{};
  auto discard = [&](int code, const char* what) {
    for (auto& b : nbufs) b.release();
    njoblist.release();
    return fail(c, code, what);
  };
  hipStream_t s = c->stream;
  int k = 0;
  auto put = [&](const void* src, size_t bytes) -> const void* {
    if (e != hipSuccess || k >= (int)nbufs.size()) {
      if (e == hipSuccess) e = hipErrorOutOfMemory;
      return nullptr;
    }
    DevBuf& b = nbufs[k++];
    e = b.ensure(bytes + 64);  // padded: the word readers (load_u32u, copy_bytes) read up to 8 bytes past a string
    if (e == hipSuccess && bytes) e = hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice);
    return b.p;
  };
  std::vector<uint32_t> top_ph;
  uint32_t n_ph1 = 0;
  const char* ferr = fill_dprogram(P, np, put, top_ph, n_ph1);
  if (e != hipSuccess) return discard(e == hipErrorOutOfMemory ? GI_ENOMEM : GI_ENODEV, "ruleset upload failed");
  if (ferr) return discard(GI_EINVAL, ferr);
  // k_scan plan: LDS jobs that fit the small image go to the 2-per-CU launch,
  // the rest (big images, global-table automata) to the 1-per-CU launch.
  std::vector<uint32_t> jl[3];
  const bool force_hbm = getenv("GI_SCAN_HBM") && atoi(getenv("GI_SCAN_HBM")) > 0;  // debugging
  for (uint32_t j = 0; j < P.jobs.size(); j++)
    jl[(force_hbm || !P.jobs[j].lds) ? 2 : P.jobs[j].big ? 1 : 0].push_back(j);
  // by stream, so k_scan can count each stream's queue words once per launch
  for (auto& l : jl)
    std::stable_sort(l.begin(), l.end(), [&](uint32_t a, uint32_t b) { return P.jobs[a].stream < P.jobs[b].stream; });
  std::vector<uint32_t> all(jl[0]);
  all.insert(all.end(), jl[1].begin(), jl[1].end());
  all.insert(all.end(), jl[2].begin(), jl[2].end());
  std::vector<uint32_t> ids;
  for (const DRule& r : P.rules)
    if (r.id > 0 && !(r.flags & RF_CHILD)) ids.push_back((uint32_t)r.id);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  DevBuf nidbuf;
  if (upload(&njoblist, all, s) != hipSuccess || upload(&nidbuf, ids, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    nidbuf.release();
    return discard(GI_ENOMEM, "scan plan upload failed");
  }
  DevBuf nprog;
  if (nprog.ensure(sizeof(DProgram)) != hipSuccess || hipMemcpy(nprog.p, &np, sizeof(DProgram), hipMemcpyHostToDevice) != hipSuccess) {
    nprog.release();
    nidbuf.release();
    return discard(GI_ENOMEM, "program upload failed");
  }
  for (int b = 0; b < 2; b++) {
    nscan.jobs[b] = (const uint32_t*)njoblist.p + (b ? jl[0].size() : 0);
    nscan.n_jobs[b] = (uint32_t)jl[b].size();
    nscan.lds[b] = b ? std::max<uint32_t>(P.max_big_img_bytes, 16) : std::max<uint32_t>(P.max_img_bytes, 16);
    scan_allow_lds(nscan.lds[b]);
    nscan.blocks[b] = scan_resident_blocks(nscan.lds[b]);
    nscan.rpl[b] = 4;
  }
  nscan.global_jobs = (const uint32_t*)njoblist.p + jl[0].size() + jl[1].size();
  nscan.n_global = (uint32_t)jl[2].size();
  nscan.blocks[2] = scan_resident_blocks(16);
  nscan.mode = getenv("GI_SCAN_MODE") ? (uint32_t)atoi(getenv("GI_SCAN_MODE")) : 0u;
  // commit: the context now runs the new program; the old buffers go
  for (auto& b : c->pbufs) b.release();
  c->joblist.release();
  c->tally_idbuf.release();
  c->progdev.release();
  c->progdev = nprog;
  c->pbufs.swap(nbufs);
  c->joblist = njoblist;
  c->tally_idbuf = nidbuf;
  c->tally_ids.swap(ids);
  c->prog = np;
  c->scan = nscan;
  c->rs = rs;
  c->staged = false;
  c->ran = false;
  return GI_OK;
}

int gi_ctx_create(const gi_ruleset* rs, int device, uint32_t matched_cap, gi_ctx** out) {
  if (!rs || !out) return GI_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return GI_ENODEV;
  auto* c = new gi_ctx();
  c->rs = rs;
  c->device = device;
  c->mcap = matched_cap ? matched_cap : 64;
  c->diag_on = getenv("GI_DIAG") && atoi(getenv("GI_DIAG")) > 0;
  c->prof_on = getenv("GI_PROF") && atoi(getenv("GI_PROF")) > 0;
  if (getenv("GI_EVAL_WAVE_FIELDS")) c->wave_fields = (uint32_t)atoi(getenv("GI_EVAL_WAVE_FIELDS"));  // A/B, 0: off
  if (getenv("GI_EVAL_WAVE_RULES")) c->wave_rules = (uint32_t)atoi(getenv("GI_EVAL_WAVE_RULES"));
  c->stage_prof = getenv("GI_STAGE_PROF") && atoi(getenv("GI_STAGE_PROF")) > 0;
  if (getenv("GI_BPARSE_WAVE")) c->bparse_wave = (uint32_t)atoi(getenv("GI_BPARSE_WAVE"));
  if (getenv("GI_BPARSE_WIN")) c->bparse_win = (uint32_t)std::min(65536, std::max(2048, atoi(getenv("GI_BPARSE_WIN")))) & ~15u;
  if (getenv("GI_BPARSE_LDS")) c->bparse_lds = (uint32_t)std::min(65536, std::max(0, atoi(getenv("GI_BPARSE_LDS"))));
  if (getenv("GI_CHUNK_POOL_WORDS")) c->chunk_pool_words = std::max(1e6, atof(getenv("GI_CHUNK_POOL_WORDS")));
  if (getenv("GI_CHUNK_CAP_BYTES")) c->chunk_cap_bytes = std::max<uint64_t>(1ull << 16, strtoull(getenv("GI_CHUNK_CAP_BYTES"), nullptr, 10));
  c->stop_after = getenv("GI_STOP_AFTER") ? atoi(getenv("GI_STOP_AFTER")) : 0;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipEventCreate(&c->evs[0]);
  if (e == hipSuccess) e = hipEventCreate(&c->evs[1]);
  if (e == hipSuccess) e = hipEventCreate(&c->evs[2]);
  for (int k = 0; k <= GI_MAX_LAUNCHES && e == hipSuccess; k++) e = hipEventCreate(&c->log.ev[k]);
  if (e != hipSuccess) {
    delete c;
    return GI_ENODEV;
  }
  const int rc = load_program(c, rs);
  if (rc != GI_OK) {
    gi_ctx_free(c);
    return rc;
  }
  if (c->stop_after)
    fprintf(stderr, "scan plan: small %u jobs lds %u blocks %u | big %u jobs lds %u blocks %u | hbm %u jobs blocks %u\n",
            c->scan.n_jobs[0], c->scan.lds[0], c->scan.blocks[0], c->scan.n_jobs[1], c->scan.lds[1],
            c->scan.blocks[1], c->scan.n_global, c->scan.blocks[2]);
  *out = c;
  return GI_OK;
}

int gi_ctx_set_capture_cap(gi_ctx* c, uint32_t records, uint32_t bytes) {
  if (!c || records == 0 || records > (1u << 16) || bytes > (1u << 30)) return GI_EINVAL;
  c->crcap = records;
  c->cbcap = bytes;
  return GI_OK;
}

int gi_ctx_swap_ruleset(gi_ctx* c, const gi_ruleset* rs) {
  if (!c || !rs) return GI_EINVAL;
  (void)hipSetDevice(c->device);
  if (hipStreamSynchronize(c->stream) != hipSuccess) return GI_ENODEV;
  const int rc = load_program(c, rs);
  if (rc != GI_OK) return fail(c, rc, "ruleset upload failed");
  return GI_OK;
}

void gi_ctx_free(gi_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& b : c->pbufs) b.release();
  c->prof.release();
  for (DevBuf* b : {&c->caprec, &c->capbytes, &c->data, &c->reqs, &c->hdrs, &c->layout, &c->scratch, &c->verdicts, &c->matched, &c->tally, &c->tally_ext, &c->tally_idbuf,
                    &c->hits, &c->vmap, &c->hset, &c->blist, &c->joblist, &c->txslots, &c->bcounts, &c->boffs, &c->items, &c->igm, &c->lscratch, &c->pool, &c->qblk,
                    &c->ctr, &c->slow, &c->slow_bytes, &c->det, &c->det_bytes, &c->long_list, &c->long_buf, &c->wlist, &c->pend, &c->plist, &c->dmemo_keys, &c->dmemo_info,
                    &c->eorder, &c->ekey, &c->hdkeys, &c->hdinfo, &c->hdref, &c->cappool, &c->progdev})
    b->release();
  for (auto& ev : c->evs)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : c->log.ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->lay_host) (void)hipHostFree(c->lay_host);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* gi_last_error(const gi_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* gi_ctx_stream(gi_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gi_host_register(gi_ctx* c, void* p, size_t n) {
  if (!c || !p || !n) return GI_EINVAL;
  (void)hipSetDevice(c->device);
  const hipError_t e = hipHostRegister(p, n, hipHostRegisterDefault);
  return e == hipSuccess ? GI_OK : hip_fail(c, e, "hipHostRegister");
}

int gi_host_unregister(gi_ctx* c, void* p) {
  if (!c || !p) return GI_EINVAL;
  (void)hipSetDevice(c->device);
  const hipError_t e = hipHostUnregister(p);
  return e == hipSuccess ? GI_OK : hip_fail(c, e, "hipHostUnregister");
}

}  // extern "C"
// One request's scratch layout and capacities (lengths only): its region in
// the batch scratch (ReqLayout), the phase-A item / hit-set sizes, and the
// batch totals it adds to.  Shared by gi_stage_batch and the CPU baseline.
struct LayoutSizes {
  uint64_t region, vmap, hset;
  uint64_t capb;                    // capture area (DBatch.cappool), outside the region
  uint64_t items, raw, body, post;  // phase-A items, bytes without / of the body, body fields
  bool mp;                          // multipart body
};
struct LayoutAcc {
  uint64_t items_cap = 0, raw_total = 0, raw_body = 0, post_total = 0, max_req_bytes = 0;
  uint32_t n_mp_body = 0, max_cap_t = 64;
};
static const char* request_layout(const Program& PG, uint32_t cap_ws_words, uint32_t cap_groups, const gi_batch* in,
                                  uint32_t r, ReqLayout& L, LayoutSizes& z, LayoutAcc& a) {
  const uint32_t n_single_items = (uint32_t)__builtin_popcount(PG.item_singles);
  z.mp = false;
  const gi_request& q = in->reqs[r];
  const gi_span* sp[6] = {&q.method, &q.uri, &q.proto, &q.body, &q.remote_addr, &q.server_name};
  for (auto* s : sp)
    if (s->off + s->len > in->data_len) return "request span out of range";
  if ((uint64_t)q.hdr_begin + q.hdr_count > in->n_headers) return "header range out of range";
  uint64_t maxv = std::max<uint64_t>({(uint64_t)q.uri.len * 3 + 2, (uint64_t)q.method.len + q.uri.len + q.proto.len + 2,
                                      (uint64_t)q.body.len, (uint64_t)q.server_name.len, 64});
  uint64_t cookie = 0, ncookie = 0, hdr_bytes = 0, hname_bytes = 0;
  bool multipart = false, hname_high = false;
  for (uint32_t h = 0; h < q.hdr_count; h++) {
    const gi_header& hd = in->headers[q.hdr_begin + h];
    if (hd.name.off + hd.name.len > in->data_len || hd.value.off + hd.value.len > in->data_len)
      return "header span out of range";
    maxv = std::max<uint64_t>(maxv, std::max(hd.name.len, hd.value.len));
    hdr_bytes += hd.name.len + hd.value.len;
    hname_bytes += hd.name.len;
    if (!PG.dyn_sites.empty())
      for (uint32_t k = 0; k < hd.name.len && !hname_high; k++) hname_high = in->data[hd.name.off + k] >= 0x80;
    if (hd.name.len == 12 && strncasecmp((const char*)in->data + hd.name.off, "content-type", 12) == 0) {
      const char* hv = (const char*)in->data + hd.value.off;
      for (uint32_t k = 0; k + 9 <= hd.value.len && !multipart; k++)
        multipart = strncasecmp(hv + k, "multipart", 9) == 0;
    }
    if (hd.name.len == 6) {
      const uint8_t* nm = in->data + hd.name.off;
      bool ck = true;
      const char* lit = "cookie";
      for (int i = 0; i < 6; i++)
        if ((nm[i] | 0x20) != lit[i]) ck = false;
      if (ck) {
        cookie += hd.value.len;
        ncookie++;
      }
    }
  }
  // ARGS_POST fields a body can yield: urlencoded <= '&' + 1; JSON <=
  // ',' + 2 '[' + '{' + 1 (elements past the first of a container need a
  // comma, and each non-empty array adds its own count entry)
  uint64_t post_fields = 0;
  if (q.body.len) {
    const uint8_t* bd = in->data + q.body.off;
    uint64_t seps = 0, nls = 0;
    for (uint32_t k = 0; k < q.body.len; k++) {
      const uint8_t ch = bd[k];
      seps += (ch == '&') + (ch == ',') + 2 * (ch == '[') + (ch == '{');
      nls += ch == '\n';
    }
    post_fields = std::min<uint64_t>(seps + 2, q.body.len / 2 + 2);
    {  // XML (kernels.hip parse_xml): one field per attribute ('=' or a bare name) and text token
      uint32_t k = 0;
      while (k < q.body.len && (bd[k] == ' ' || bd[k] == '\t' || bd[k] == '\n' || bd[k] == '\r')) k++;
      if (k < q.body.len && bd[k] == '<') {
        uint64_t lt = 0, sp = 0;
        for (uint32_t j = 0; j < q.body.len; j++) {
          lt += bd[j] == '<';
          sp += bd[j] == ' ' || bd[j] == '\t' || bd[j] == '\n' || bd[j] == '\r';
        }
        post_fields = std::max<uint64_t>(post_fields, 2 * lt + sp + 2);
      }
    }
    // multipart (kernels.hip parse_multipart): a part spends >= 2 lines on
    // its delimiter and header end and yields <= 3 entries + 1 per header line
    if (multipart) post_fields += nls + 8;
    a.n_mp_body += multipart ? 1 : 0;
    z.mp = multipart;
  }
  uint64_t cap_f = q.hdr_count + (q.uri.len / 2 + 2) + (cookie / 2 + 2 * ncookie) + post_fields;
  // + REMOTE_PORT; the URI: REQUEST_LINE, decoded path / host / userinfo, String() (<= 3x each part)
  uint64_t cap_b = 12ull * q.uri.len + q.method.len + q.proto.len + q.body.len + 96 + 16;
  // multipart: canonical keys, joined continuation lines, "Key: value"
  // strings and unescaped parameters are each at most the part header
  // bytes; sizes 24 B per part
  if (multipart) cap_b += 4ull * q.body.len + 1024;
  // XML (a ctl can pick it for any body): decoded texts <= the body, the error message
  if (q.body.len) cap_b += q.body.len + 1024;
  {  // a JSON-looking body: room for the flattened "json.a.b" keys + parser stack
    const uint8_t* bd = in->data + q.body.off;
    uint32_t k = 0;
    while (k < q.body.len && (bd[k] == ' ' || bd[k] == '\t' || bd[k] == '\n' || bd[k] == '\r')) k++;
    // kernels.hip parse_json_body: flattened bytes <= 4n + 1024, one
    // transient allocation <= that again + n, parser stack 1048 B
    if (k < q.body.len && (bd[k] == '{' || bd[k] == '[')) cap_b += 8ull * q.body.len + 4200;
  }
  cap_b += 8 * (cap_f + 12) + 8;  // k_eval's kind index, built for phase 1 and again after the body parse
  uint64_t cap_t = 3 * maxv + 64 + (q.body.len ? 8 * 64 : 0);  // k_body: 64 lane slots of 3x + 8 B
  uint64_t cap_mt = 2 * maxv + 512;
  if (cap_f > 0xFFFFFFFFull || cap_b > 0xFFFFFFFFull || cap_t > 0xFFFFFFFFull || cap_mt > 0xFFFFFFFFull)
    return "request too large";
  // phase-A items: at most both sides of every field (GET args, headers,
  // cookies; POST args appear after phase 1) plus the filtered singles
  const uint64_t pre_body_fields = q.hdr_count + (q.uri.len / 2 + 2) + (cookie / 2 + 2 * ncookie);
  z.items = 2 * (pre_body_fields + (PG.body_access ? post_fields : 0)) + n_single_items;
  z.post = PG.body_access ? post_fields : 0;
  z.raw = (uint64_t)q.method.len + q.uri.len + q.proto.len + hdr_bytes;
  z.body = q.body.len;
  a.items_cap += z.items;
  a.post_total += PG.body_access ? post_fields : 0;
  a.raw_total += (uint64_t)q.method.len + q.uri.len + q.proto.len + hdr_bytes;
  a.raw_body += q.body.len;
  a.max_req_bytes = std::max<uint64_t>(a.max_req_bytes, (uint64_t)q.method.len + q.uri.len + q.proto.len + hdr_bytes + q.body.len);
  a.max_cap_t = (uint32_t)std::max<uint64_t>(a.max_cap_t, cap_t);
  
  L.vmap_bits = (uint32_t)(2 * cap_f);
  z.vmap = (2 * cap_f + 31) & ~31ull;
  {  // exact hit set (kernels.hip hset_insert): ~one key per phase-A item; a fuller table
     // only sends the request back to re-evaluation (exact either way)
    uint64_t amps = 1;
    const uint8_t* u = in->data + q.uri.off;
    for (uint32_t k = 0; k < q.uri.len; k++) amps += u[k] == '&';
    const uint64_t est = 2 * (amps + q.hdr_count + 2 * ncookie + cookie / 8 + (PG.body_access ? post_fields : 0)) +
                         n_single_items;
    uint64_t cap = 16;
    while (cap < est && cap < (1ull << 16)) cap <<= 1;
    L.hset_mask = PG.streams.empty() ? 0u : (uint32_t)(cap - 1);
    z.hset = PG.streams.empty() ? 0 : (cap + 1 + 3) & ~3ull;
  }
  // dynamic TX area (macro-key setvars): the executions each site can reach on
  // this request and the bytes they can store (gi_program.h DDynSite)
  uint64_t dyn_e = 0, dyn_b = 0;
  for (const DDynSite& ds : PG.dyn_sites) {
    if (ds.dead) continue;  // an unreachable rule's setvar never runs
    const uint64_t raw_all = (uint64_t)q.method.len + q.uri.len + q.proto.len + hdr_bytes + q.body.len;
    uint64_t ex = ds.mm, src = 0;
    if (!ds.no_targets) {
      ex = (uint64_t)ds.mm * (ds.nsingles + (uint64_t)(ds.hdr_names + ds.hdr_vals) * q.hdr_count + (uint64_t)ds.other_coll * cap_f);
      src = (uint64_t)ds.mm * (ds.nsingles * maxv + (uint64_t)ds.hdr_names * hname_bytes +
                               (uint64_t)ds.hdr_vals * (hdr_bytes - hname_bytes) + (uint64_t)ds.other_coll * (raw_all + cap_b));
    }
    const bool ascii_src = !ds.hdr_vals && !ds.other_coll && !ds.nsingles && !hname_high;
    const uint64_t g = ascii_src ? ds.g_ascii : ds.g_any;
    dyn_e += ex;
    dyn_b += ex * (ds.lit + ds.fixed + 32ull * ds.n_mvname) + g * (ds.n_val + ds.n_mvname) * src +
             ex * ds.n_big * std::max(cap_t, cap_mt);
  }
  if (dyn_e > 0xFFFFFFFFull || dyn_b > 0xFFFFFFFFull) return "request too large (dynamic TX keys)";
  L.dyn_cap = PG.dyn_sites.empty() ? 0u : (uint32_t)dyn_e;
  L.dyn_capb = PG.dyn_sites.empty() ? 0u : (uint32_t)((dyn_b + 15) & ~15ull);
  L.cap_f = (uint32_t)cap_f;
  L.cap_b = (uint32_t)cap_b;
  L.cap_t = (uint32_t)cap_t;
  L.cap_mt = (uint32_t)cap_mt;
  uint64_t sz = GI_REQHDR_BYTES + cap_f * 32 + ((uint64_t)PG.n_slots * GI_SLOT_BYTES + 15) / 16 * 16 + GI_RM_BYTES + (cap_b + 15) / 16 * 16 +
                2 * ((cap_t + 15) / 16 * 16) + 2 * ((cap_mt + 15) / 16 * 16);
  if (!PG.dyn_sites.empty()) sz += 16 + 32ull * L.dyn_cap + L.dyn_capb;  // kernels.hip DynHdr + DynEnt[] + bytes
  // observable captures (kernels.hip region_of): workspace + one value buffer
  // per group, in the chunk's capture pool rather than the region
  z.capb = cap_ws_words ? (4ull * cap_ws_words + 15) / 16 * 16 + (uint64_t)cap_groups * ((cap_t + 15) / 16 * 16) : 0;
  // matched-variable state (kernels.hip MvState): header, entries, value
  // arena, MATCHED_VAR copy, name buffer
  if (PG.mv_used) {
    // MATCHED_VARS of one rule: a value per field (transformed: <= cap_t... the
    // arena holds what phase B copies), plus the TX entries a TX target can
    // match -- the static slots (values <= the longest setvar literal or a
    // macro expansion) and the run-time keys
    const uint64_t e = cap_f + 16 + PG.n_slots + L.dyn_cap;
    // TX values: a string a slot holds lives in the TX string arena (cap_mt
    // bytes in all), the string pool (one literal per slot), the dynamic area
    // (dyn_capb) or is a formatted integer -- so their sum, not n_slots x the
    // largest, bounds one rule's MATCHED_VARS copies of them; a capture group
    // (TX.0 .. TX.<cap_groups - 1>) holds at most cap_t bytes of its value buffer
    const uint64_t tx_vals = cap_mt + (uint64_t)PG.n_slots * (PG.max_tx_lit + 24) + (uint64_t)cap_groups * cap_t;
    const uint64_t ab = cap_b + cap_mt + L.dyn_capb + 40ull * (PG.n_slots + L.dyn_cap) + tx_vals;
    if (e > 0xFFFFFFFFull || ab > 0xFFFFFFFFull) return "request too large (matched variables)";
    L.mv_cap_e = (uint32_t)e;
    L.mv_cap_a = (uint32_t)((ab + 15) & ~15ull);
    sz += 64 + e * 32 + L.mv_cap_a + (cap_t + 15) / 16 * 16 + (cap_mt + 15) / 16 * 16;
  }
  z.region = (sz + 63) / 64 * 64;
  return nullptr;
}

extern "C" {
int gi_stage_batch(gi_ctx* c, const gi_batch* in) {
  if (!c || !in) return GI_EINVAL;
  if (in->n_req && (!in->reqs || !in->data)) return fail(c, GI_EINVAL, "null batch arrays");
  (void)hipSetDevice(c->device);
  auto t0 = std::chrono::steady_clock::now();
  auto t_sizes = t0, t_plan = t0;
  const uint32_t n = in->n_req;
  // validate spans and lay out per-request scratch (lengths only)
  // the layout lives in a page-locked host buffer of the ctx (reused), so its
  // H2D is a DMA copy
  if (c->lay_host_cap < n) {
    if (c->lay_host) (void)hipHostFree(c->lay_host);
    c->lay_host = nullptr;
    c->lay_host_cap = 0;
    if (hipHostMalloc((void**)&c->lay_host, std::max<size_t>(n, 1) * sizeof(ReqLayout)) == hipSuccess) c->lay_host_cap = n;
    else c->lay_host = nullptr;
  }
  std::vector<ReqLayout> lay_v(c->lay_host ? 0 : n);
  ReqLayout* lay = c->lay_host ? c->lay_host : lay_v.data();
  uint64_t off = 0, items_cap = 0, raw_total = 0, raw_body = 0, post_total = 0, vmap_bits = 0, max_req_bytes = 0;
  uint64_t hset_words = 0;
  uint32_t n_mp_body = 0;
  uint32_t max_cap_t = 64;
  const Program& PG = c->rs->prog;
  // per-request sizes (in parallel on the host cores for large batches),
  // then the running offsets (region, value map, hit set) in one serial pass
  using Sizes = LayoutSizes;
  using Acc = LayoutAcc;
  std::vector<Sizes> sizes(n);
  for (auto& z : sizes) z.mp = false;
  auto size_one = [&](uint32_t r, Acc& a) -> const char* {
    return request_layout(PG, c->prog.cap_ws_words, c->prog.cap_groups, in, r, lay[r], sizes[r], a);
  };
  {
    const uint32_t nt = n >= 65536 ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
    std::vector<Acc> acc(nt);
    std::vector<const char*> errs(nt, nullptr);
    auto work = [&](uint32_t k) {
      const uint32_t lo = (uint32_t)((uint64_t)n * k / nt), hi = (uint32_t)((uint64_t)n * (k + 1) / nt);
      for (uint32_t r = lo; r < hi && !errs[k]; r++) errs[k] = size_one(r, acc[k]);
    };
    if (nt == 1) {
      work(0);
    } else {
      // a thread the system refuses (pid / thread limits) must not throw across
      // the C ABI: its slice runs on the calling thread instead
      std::vector<std::thread> th;
      std::vector<uint32_t> inline_slices;
      for (uint32_t k = 0; k < nt; k++) {
        try {
          th.emplace_back(work, k);
        } catch (...) {
          inline_slices.push_back(k);
        }
      }
      for (uint32_t k : inline_slices) work(k);
      for (auto& x : th) x.join();
    }
    for (uint32_t k = 0; k < nt; k++)
      if (errs[k]) return fail(c, GI_EINVAL, errs[k]);
    t_sizes = std::chrono::steady_clock::now();
    for (const Acc& a : acc) {
      items_cap += a.items_cap;
      raw_total += a.raw_total;
      raw_body += a.raw_body;
      post_total += a.post_total;
      max_req_bytes = std::max(max_req_bytes, a.max_req_bytes);
      n_mp_body += a.n_mp_body;
      max_cap_t = std::max(max_cap_t, a.max_cap_t);
    }
    for (uint32_t r = 0; r < n; r++) {
      ReqLayout& L = lay[r];
      L.base = off;
      L.vmap_bit = vmap_bits;
      L.hset_word = hset_words;
      off += sizes[r].region;
      vmap_bits += sizes[r].vmap;
      hset_words += sizes[r].hset;
    }
  }
  t_plan = std::chrono::steady_clock::now();
  hipError_t e = hipSuccess;
  hipStream_t s = c->stream;
  // +16: word-granular readers may touch up to 7 bytes past a value's end
  if ((e = c->data.ensure(std::max<uint64_t>(in->data_len + 16, 16))) != hipSuccess) return hip_fail(c, e, "alloc data");
  if ((e = c->reqs.ensure(std::max<size_t>(n * sizeof(gi_request), 16))) != hipSuccess) return hip_fail(c, e, "alloc reqs");
  if ((e = c->hdrs.ensure(std::max<size_t>(in->n_headers * sizeof(gi_header), 16))) != hipSuccess)
    return hip_fail(c, e, "alloc headers");
  if ((e = c->layout.ensure(std::max<size_t>(n * sizeof(ReqLayout), 16))) != hipSuccess) return hip_fail(c, e, "alloc layout");
  if ((e = c->scratch.ensure(std::max<uint64_t>(off + 64, 64))) != hipSuccess) return hip_fail(c, e, "alloc scratch");
  if ((e = c->verdicts.ensure(std::max<size_t>(n * sizeof(gi_verdict), 16))) != hipSuccess)
    return hip_fail(c, e, "alloc verdicts");
  if ((e = c->matched.ensure(std::max<size_t>((size_t)n * c->mcap * 4, 16))) != hipSuccess)
    return hip_fail(c, e, "alloc matched");
  c->cap_on = c->prog.cap_ws_words != 0;
  if (c->cap_on) {
    if ((e = c->caprec.ensure(std::max<size_t>(16ull * n * c->crcap, 16))) != hipSuccess) return hip_fail(c, e, "alloc capture records");
    if ((e = c->capbytes.ensure(std::max<size_t>((size_t)n * c->cbcap, 16))) != hipSuccess) return hip_fail(c, e, "alloc capture bytes");
  }
  c->staged_crcap = c->crcap;
  c->staged_cbcap = c->cbcap;
  if ((e = c->tally.ensure(sizeof(gi_tally))) != hipSuccess) return hip_fail(c, e, "alloc tally");
  if ((e = c->tally_ext.ensure(4ull * (GI_SCORE_BINS + c->tally_ids.size()))) != hipSuccess)
    return hip_fail(c, e, "alloc detail tally");
  if ((e = c->txslots.ensure(std::max<uint64_t>((uint64_t)GI_SLOT_BYTES * PG.n_slots * n, 64))) != hipSuccess)
    return hip_fail(c, e, "alloc tx slots");
  c->hit_words = (PG.n_hit_slots + 31) / 32;
  c->vmap_words = vmap_bits;  // one u32 slot signature per (field, side): bit (slot % 32) of each slot it hit
  c->hset_words = hset_words;
  if ((e = c->hset.ensure(std::max<uint64_t>(4 * hset_words, 16))) != hipSuccess) return hip_fail(c, e, "alloc hit sets");
  // Request chunks: consecutive requests while the chunk's queue-pool
  // estimate (the formula sizing the pool below) stays within
  // chunk_pool_words; each chunk runs the whole pipeline (gi_run_staged).
  const double pf = pool_factor_env();
  auto pool_est = [&](uint64_t nn, uint64_t raw, uint64_t body, uint64_t post) {
    return pf * (1024.0 * nn + 8.0 * raw + (post ? 24.0 * body : 0.0));
  };
  struct ChunkSum {
    uint64_t n = 0, raw = 0, body = 0, post = 0, items = 0, capb = 0;
  };
  std::vector<ChunkSum> csum;
  c->chunks.clear();
  {
    ChunkSum cs;
    uint32_t r0 = 0;
    for (uint32_t r = 0; r < n; r++) {
      const Sizes& z = sizes[r];
      if (cs.n && (pool_est(cs.n + 1, cs.raw + z.raw, cs.body + z.body, cs.post + z.post) > c->chunk_pool_words ||
                   cs.capb + z.capb > c->chunk_cap_bytes)) {
        c->chunks.push_back({r0, (uint32_t)cs.n, 0, 0, 0});
        csum.push_back(cs);
        cs = ChunkSum();
        r0 = r;
      }
      cs.n++;
      cs.raw += z.raw;
      cs.body += z.body;
      cs.post += z.post;
      cs.items += z.items;
      lay[r].cap_off = cs.capb;  // chunk-relative: every chunk reuses the pool
      cs.capb += z.capb;
    }
    if (cs.n || c->chunks.empty()) {
      c->chunks.push_back({r0, (uint32_t)cs.n, 0, 0, 0});
      csum.push_back(cs);
    }
  }
  // k_body's work lists: per chunk, the requests with a body, longest first (one wave each)
  std::vector<uint32_t> blist;
  for (auto& ch : c->chunks) {
    ch.blist_off = (uint32_t)blist.size();
    for (uint32_t r = 0; r < ch.n; r++)
      if (in->reqs[ch.r0 + r].body.len) {
        blist.push_back(r);  // chunk-local index
        ch.n_mp += sizes[ch.r0 + r].mp ? 1u : 0u;
      }
    ch.n_body = (uint32_t)blist.size() - ch.blist_off;
    std::stable_sort(blist.begin() + ch.blist_off, blist.end(), [&](uint32_t x, uint32_t y) {
      return in->reqs[ch.r0 + x].body.len > in->reqs[ch.r0 + y].body.len;
    });
  }
  c->n_body = (uint32_t)blist.size();
  c->n_mp_body = n_mp_body;
  if ((e = upload(&c->blist, blist, s)) != hipSuccess) return hip_fail(c, e, "alloc body list");
  // per-chunk maxima of the phase-A capacities
  ChunkSum cmax;
  for (const ChunkSum& cs : csum) {
    cmax.n = std::max(cmax.n, cs.n);
    cmax.items = std::max(cmax.items, cs.items);
    cmax.capb = std::max(cmax.capb, cs.capb);
  }
  if ((e = c->cappool.ensure(std::max<uint64_t>(cmax.capb + 64, 64))) != hipSuccess) return hip_fail(c, e, "alloc capture pool");
  if ((e = c->vmap.ensure(std::max<uint64_t>(4 * c->vmap_words, 16))) != hipSuccess) return hip_fail(c, e, "alloc value map");
  if ((e = c->hits.ensure(std::max<size_t>((size_t)c->hit_words * n * 4, 16))) != hipSuccess)
    return hip_fail(c, e, "alloc hits");
  if (!PG.streams.empty()) {
    // phase A: items, per-lane transformation scratch, queue pool + blocks,
    // slow list.  Pool / slow-list overflow only voids the phase-A bits of the
    // requests concerned (k_eval then evaluates their rules in full).
    const uint32_t cb = (uint32_t)((cmax.n + 255) / 256);
    const uint32_t ns = (uint32_t)PG.streams.size();
    c->items_cap = std::max<uint64_t>(cmax.items, 1);
    // header dedup table: a power of two >= the chunk's items (<= 2^24 entries, 16 B each)
    c->hdmask = 0;
    static const bool hd_env = !(getenv("GI_DEDUP") && atoi(getenv("GI_DEDUP")) == 0);
    if (hd_env && PG.item_sides[FK_HEADER] && cmax.n >= 4096) {
      uint64_t cap = 1024;
      while (cap < cmax.items && cap < (1ull << 24)) cap <<= 1;
      if ((e = c->hdkeys.ensure(8 * cap)) != hipSuccess) return hip_fail(c, e, "alloc header dedup table");
      if ((e = c->hdinfo.ensure(8 * cap)) != hipSuccess) return hip_fail(c, e, "alloc header dedup table");
      if ((e = c->hdref.ensure(std::max<uint64_t>(8ull * in->n_headers, 16))) != hipSuccess)
        return hip_fail(c, e, "alloc header dedup refs");
      c->hdmask = (uint32_t)(cap - 1);
    }
    c->lcap = (std::min<uint32_t>(max_cap_t, 4096) + 15) & ~15u;
    // chunked reservations leave at most one partial chunk per (k_stream
    // wave, launch) unused: both capacities carry that slack
    const uint64_t waves = (uint64_t)GI_STREAM_GRID * 5;
    c->qcap = (uint32_t)std::min<uint64_t>(c->items_cap / 64 + 8, 0xFFFFFFFull);  // item-waves
    uint64_t pool_max = 0, slow_max = 0, long_max = 0, det_max = 0, detb_max = 0;
    for (const ChunkSum& cs : csum) {
      pool_max = std::max<uint64_t>(pool_max, (uint64_t)pool_est(cs.n, cs.raw, cs.body, cs.post));
      slow_max = std::max<uint64_t>(slow_max, 4ull * cs.n + 4096 + cs.post / 4);
      long_max = std::max<uint64_t>(long_max, ((cs.raw + cs.body) / GI_LONG_MIN + 16) * 2ull * ns);
      // @detectSQLi/@detectXSS candidates: an item lists its unchanged value once and
      // each differently transformed output once per detect stream: 2 per item covers the common case
      const uint64_t dc = std::min<uint64_t>(std::min<uint64_t>(2ull * cs.items, 24ull * cs.n + 2ull * cs.post) + 4096,
                                             0x7FFFFFFFull);
      det_max = std::max(det_max, dc);
      detb_max = std::max<uint64_t>(detb_max, 3ull * (cs.raw + cs.body) + 16ull * dc);
    }
    c->pool_cap = std::min<uint64_t>(pool_max + waves * GI_PCHUNK + 4096, 0x3FFFFFFF0ull);  // qblk cell indices: 2^32 x 16 B
    c->slow_cap = (uint32_t)std::min<uint64_t>(slow_max, 0x7FFFFFFFull);
    c->slow_bytes_cap = 64ull * c->slow_cap;
    if ((e = c->bcounts.ensure(4ull * cb * GI_NCLS)) != hipSuccess) return hip_fail(c, e, "alloc bcounts");
    if ((e = c->boffs.ensure(4ull * cb * GI_NCLS)) != hipSuccess) return hip_fail(c, e, "alloc boffs");
    if ((e = c->items.ensure(32ull * c->items_cap)) != hipSuccess) return hip_fail(c, e, "alloc items");
    if ((e = c->igm.ensure(8ull * c->items_cap)) != hipSuccess) return hip_fail(c, e, "alloc item filter masks");
    if ((e = c->lscratch.ensure((uint64_t)GI_STREAM_GRID * 64 * 2 * c->lcap + 64)) != hipSuccess)
      return hip_fail(c, e, "alloc lane scratch");
    if ((e = c->pool.ensure(4ull * c->pool_cap)) != hipSuccess) return hip_fail(c, e, "alloc queue pool");
    if ((e = c->qblk.ensure(8ull * ns * c->qcap)) != hipSuccess) return hip_fail(c, e, "alloc queue blocks");
    if ((e = c->ctr.ensure(4096 + 8ull * ((4 * GI_NCLS + 63) & ~63))) != hipSuccess) return hip_fail(c, e, "alloc counters");
    (void)ns;
    if ((e = c->slow.ensure(40ull * c->slow_cap)) != hipSuccess) return hip_fail(c, e, "alloc slow list");
    if ((e = c->slow_bytes.ensure(c->slow_bytes_cap + 16)) != hipSuccess) return hip_fail(c, e, "alloc slow bytes");
    // long values (>= GI_LONG_MIN bytes): one k_long wave per (item, stream), each
    // workgroup with two buffers of 3x the longest request (overflow: "maybe", exact)
    c->long_cap = (uint32_t)std::min<uint64_t>(long_max, 0x7FFFFFFFull);
    // The buffers are bounded by GI_LONG_BUDGET bytes in total: fewer k_long
    // workgroups when the longest request is large, and a per-buffer cap past
    // which a chain overflows ("maybe": k_eval evaluates those links, exact),
    // so one oversized request can never fail the batch's allocation.
    c->long_bufcap = std::min<uint64_t>((3ull * max_req_bytes + 1024 + 15) & ~15ull, GI_LONG_BUDGET / 2);
    c->long_grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(GI_LONG_GRID, GI_LONG_BUDGET / (2 * c->long_bufcap)));
    if ((e = c->long_list.ensure(8ull * c->long_cap)) != hipSuccess) return hip_fail(c, e, "alloc long-value list");
    if ((e = c->long_buf.ensure((uint64_t)c->long_grid * 2 * c->long_bufcap)) != hipSuccess)
      return hip_fail(c, e, "alloc long-value buffers");
    // @detectSQLi/@detectXSS candidate list (overflow: the vals' bits become "maybe", exact)
    c->det_cap = c->prog.n_det_streams ? (uint32_t)det_max : 0;
    c->det_bytes_cap = c->prog.n_det_streams ? detb_max : 0;
    if ((e = c->det.ensure(std::max<uint64_t>(32ull * c->det_cap, 64))) != hipSuccess) return hip_fail(c, e, "alloc detect list");
    // detector memo: a power of two >= 2 x the candidates (at most 2^25 slots, 24 B each)
    c->dmemo_mask = 0;
    static const bool memo_env = !(getenv("GI_DET_MEMO") && atoi(getenv("GI_DET_MEMO")) == 0);
    if (c->det_cap && memo_env) {
      uint64_t cap = 1024;
      while (cap < 2ull * c->det_cap && cap < (1ull << 25)) cap <<= 1;
      if ((e = c->dmemo_keys.ensure(8 * cap)) != hipSuccess) return hip_fail(c, e, "alloc detect memo");
      if ((e = c->dmemo_info.ensure(16 * cap)) != hipSuccess) return hip_fail(c, e, "alloc detect memo");
      c->dmemo_mask = (uint32_t)(cap - 1);
    }
    if ((e = c->det_bytes.ensure(c->det_bytes_cap + 16)) != hipSuccess) return hip_fail(c, e, "alloc detect bytes");
  }
  // k_eval -> k_eval_wave request list (its counter lives in ctr)
  if ((e = c->ctr.ensure(4096 + 8ull * ((4 * GI_NCLS + 63) & ~63))) != hipSuccess) return hip_fail(c, e, "alloc counters");
  if ((e = c->wlist.ensure(4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return hip_fail(c, e, "alloc wave list");
  if ((e = c->eorder.ensure(4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return hip_fail(c, e, "alloc eval order");
  if ((e = c->ekey.ensure(std::max<uint64_t>(n, 16))) != hipSuccess) return hip_fail(c, e, "alloc eval order keys");
  if ((e = c->pend.ensure(std::max<uint64_t>(n, 16))) != hipSuccess) return hip_fail(c, e, "alloc gate flags");
  if ((e = c->plist.ensure(4ull * std::max<uint32_t>(n, 1))) != hipSuccess) return hip_fail(c, e, "alloc gate list");
  const auto t_h2d0 = std::chrono::steady_clock::now();
  if (in->data_len) e = hipMemcpyAsync(c->data.p, in->data, in->data_len, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(c->reqs.p, in->reqs, n * sizeof(gi_request), hipMemcpyHostToDevice, s);
  if (e == hipSuccess && in->n_headers)
    e = hipMemcpyAsync(c->hdrs.p, in->headers, in->n_headers * sizeof(gi_header), hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(c->layout.p, lay, n * sizeof(ReqLayout), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "stage H2D");
  if (c->stage_prof) {
    auto ms = [&](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t_end = std::chrono::steady_clock::now();
    fprintf(stderr, "GI_STAGE_PROF n=%u chunks=%zu: sizes %.1f ms, offsets+chunks+lists %.1f ms, allocs %.1f ms, H2D %.1f ms\n",
            n, c->chunks.size(), ms(t0, t_sizes), ms(t_sizes, t_plan), ms(t_plan, t_h2d0), ms(t_h2d0, t_end));
  }
  c->n_req = n;
  c->max_body = 0;
  for (uint32_t r = 0; r < n; r++) c->max_body = std::max<uint64_t>(c->max_body, in->reqs[r].body.len);
  c->staged = true;
  c->ran = false;
  c->stats.last_scratch_bytes = off;
  c->stats.last_pa_bytes = 4ull * c->pool_cap;
  c->raw_nobody = raw_total;
  c->raw_all = raw_total + raw_body;
  c->stats.last_stage_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GI_OK;
}

int gi_run_staged(gi_ctx* c) {
  if (!c) return GI_EINVAL;
  if (!c->staged) return fail(c, GI_ESTATE, "gi_run_staged before gi_stage_batch");
  (void)hipSetDevice(c->device);
  hipError_t e = hipMemsetAsync(c->tally.p, 0, sizeof(gi_tally), c->stream);
  if (e == hipSuccess)
    e = hipMemsetAsync(c->tally_ext.p, 0, 4ull * (GI_SCORE_BINS + c->tally_ids.size()), c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "memset tally");
  DBatch B{};
  B.data = (const uint8_t*)c->data.p;
  B.reqs = (const gi_request*)c->reqs.p;
  B.headers = (const gi_header*)c->hdrs.p;
  B.n_req = c->n_req;
  B.mcap = c->mcap;
  B.scratch = (uint8_t*)c->scratch.p;
  B.cappool = (uint8_t*)c->cappool.p;
  B.prog = (const DProgram*)c->progdev.p;
  B.layout = (const ReqLayout*)c->layout.p;
  B.verdicts = (gi_verdict*)c->verdicts.p;
  B.matched = (uint32_t*)c->matched.p;
  B.caprec = c->cap_on ? (uint32_t*)c->caprec.p : nullptr;
  B.capbytes = c->cap_on ? (uint8_t*)c->capbytes.p : nullptr;
  B.crcap = c->staged_crcap;
  B.cbcap = c->staged_cbcap;
  B.tally = (unsigned long long*)c->tally.p;
  B.tally_ext = (uint32_t*)c->tally_ext.p;
  B.hits = (uint32_t*)c->hits.p;
  B.vmap = (uint32_t*)c->vmap.p;
  B.hset = (uint32_t*)c->hset.p;
  B.body_list = (const uint32_t*)c->blist.p;
  B.n_body = c->n_body;
  B.n_mp_body = c->n_mp_body;
  B.txslots = (Slot*)c->txslots.p;
  {
    // counters (bytes): [0] pool words used, [8] slow bytes used, [16] slow
    // entries, [64] item buckets {(base, count) x5, item-wave base x5, item
    // waves}, [128] debug record, [160] acct: item bytes per bucket x5, queue
    // words written per k_stream bucket x5, queue words read per k_scan launch x3
    uint8_t* cp = (uint8_t*)c->ctr.p;
    B.bcounts = (uint32_t*)c->bcounts.p;
    B.boffs = (uint32_t*)c->boffs.p;
    B.ctot = (uint32_t*)(cp + 4096);  // GI_NCLS words each
    B.cbase = (uint32_t*)(cp + 4096 + ((4 * GI_NCLS + 63) & ~63));
    B.ibk = (uint32_t*)(cp + 64);
    B.items = c->items.p;
    B.igm = (uint64_t*)c->igm.p;
    B.lscratch = (uint8_t*)c->lscratch.p;
    B.lcap = c->lcap;
    B.pool = (uint32_t*)c->pool.p;
    B.pool_cap = c->pool_cap;
    B.pool_used = (unsigned long long*)cp;
    B.qblk = (uint2*)c->qblk.p;
    B.acct = (unsigned long long*)(cp + 160);
    B.acct2 = (unsigned long long*)(cp + 336);  // 6 byte-step counters
    B.acct3 = (unsigned long long*)(cp + 384);  // 5 item counts per bucket
    B.qcap = c->qcap;
    B.slow = c->slow.p;
    B.slow_count = (uint32_t*)(cp + 16);
    B.slow_cap = c->slow_cap;
    B.slow_bytes = (uint8_t*)c->slow_bytes.p;
    B.slow_bytes_cap = c->slow_bytes_cap;
    B.slow_used = (unsigned long long*)(cp + 8);
    B.long_list = (uint2*)c->long_list.p;
    B.long_count = (uint32_t*)(cp + 40);
    B.long_cap = c->prog.n_streams ? c->long_cap : 0;
    B.long_grid = c->long_grid;
    B.long_buf = (uint8_t*)c->long_buf.p;
    B.long_bufcap = c->long_bufcap;
    B.det = c->det.p;
    B.det_count = (uint32_t*)(cp + 24);
    B.det_cap = c->det_cap;
    B.det_bytes = (uint8_t*)c->det_bytes.p;
    B.det_bytes_cap = c->det_bytes_cap;
    B.det_used = (unsigned long long*)(cp + 32);
    B.dmemo_keys = c->dmemo_mask ? (unsigned long long*)c->dmemo_keys.p : nullptr;
    B.dmemo_info = c->dmemo_mask ? (uint4*)c->dmemo_info.p : nullptr;
    B.dmemo_mask = c->dmemo_mask;
    static const uint32_t dm_min_env = getenv("GI_DET_MEMO_MIN") ? (uint32_t)atoi(getenv("GI_DET_MEMO_MIN")) : 32u;
    B.dmemo_min = dm_min_env;
    B.diag = nullptr;
    B.prof = nullptr;
    if (c->prof_on && c->prof.ensure(1024 + 24000) == hipSuccess) {
      B.prof = (unsigned long long*)c->prof.p;
      (void)hipMemsetAsync(c->prof.p, 0, 1024 + 24000, c->stream);
    }
    B.items_cap = c->items_cap;
    B.n_hit_slots = c->rs->prog.n_hit_slots;
    B.vcause = (unsigned long long*)(cp + 288);  // 6 void-cause counters
    B.dbg = (uint32_t*)(cp + 128);  // 4 words (only written by -DGI_DEBUG builds)
    const bool wave = (c->wave_fields || c->wave_rules) && c->wlist.p && cp;
    B.wlist = wave ? (uint32_t*)c->wlist.p : nullptr;
    B.wcount = wave ? (uint32_t*)(cp + 48) : nullptr;
    B.wave_fields = c->wave_fields;
    B.wave_rules = c->wave_rules;
    B.rstride = c->n_req;
    // the phase-1 gate (GI_GATE=0: one pass, bodies parsed before phase 1)
    // GI_GATE: 0 off, 1 always, unset adaptive (gi_ctx::gate_pending_share)
    static const int gate_env = getenv("GI_GATE") ? atoi(getenv("GI_GATE")) : -1;
    const bool adaptive_on = c->gate_pending_share < 0 || c->gate_pending_share <= GI_GATE_PENDING_MAX ||
                             c->stats.batches % 16 == 0;
    B.stage = 0;
    B.gate = (gate_env == 1 || (gate_env < 0 && adaptive_on)) ? 1u : 0u;
    c->gate_ran = B.gate != 0;
    B.pend = (uint8_t*)c->pend.p;
    B.plist = (uint32_t*)c->plist.p;
    B.pcount = (uint32_t*)(cp + 512);
    // k_eval's request order (GI_EVAL_ORDER=0: identity): bins + cursors at ctr[1024, 1024 + 8 * GI_EORD_BINS)
    static const bool eord_env = !(getenv("GI_EVAL_ORDER") && atoi(getenv("GI_EVAL_ORDER")) == 0);
    B.eorder = eord_env ? (uint32_t*)c->eorder.p : nullptr;
    B.eord_bins = (uint32_t*)(cp + 1024);
    B.eord_key = (uint8_t*)c->ekey.p;
    B.hdkeys = c->hdmask ? (unsigned long long*)c->hdkeys.p : nullptr;
    B.hdinfo = c->hdmask ? (unsigned long long*)c->hdinfo.p : nullptr;
    B.hdref = c->hdmask ? (uint32_t*)c->hdref.p : nullptr;
    B.hdmask = c->hdmask;
    static const uint32_t tiles_env = getenv("GI_BODY_TILES") ? (uint32_t)atoi(getenv("GI_BODY_TILES")) : 1u;
    B.body_tiles = tiles_env;
    static const uint32_t ws2_env = getenv("GI_EVAL_WAVE_STAGE2") ? (uint32_t)atoi(getenv("GI_EVAL_WAVE_STAGE2")) : 1u;
    B.wave_stage2 = ws2_env;
    B.bparse_wave = c->bparse_wave;
    static const uint32_t mpw_env = getenv("GI_MP_WAVE") ? (uint32_t)atoi(getenv("GI_MP_WAVE")) : 1u;
    B.mp_wave = mpw_env;
    B.bparse_lds = c->bparse_wave ? c->bparse_win
                                  : (uint32_t)std::min<uint64_t>(c->bparse_lds, (c->max_body + 15) & ~15ull);
  }
  (void)hipEventRecord(c->ev0, c->stream);
  if (c->ctr.p) {
    e = hipMemsetAsync(c->ctr.p, 0, c->ctr.cap, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset counters");
  }
  if (c->hit_words) {
    e = hipMemsetAsync(c->hits.p, 0, (size_t)c->hit_words * c->n_req * 4, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset hits");
  }
  if (c->vmap_words) {
    e = hipMemsetAsync(c->vmap.p, 0, 4 * c->vmap_words, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset value map");
  }
  if (c->hset_words) {
    e = hipMemsetAsync(c->hset.p, 0, 4 * c->hset_words, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset hit sets");
  }
  // the request chunks (gi_stage_batch), one full pipeline pass each; the
  // phase-A counters [0, 128) of ctr restart per chunk, the accounting ones
  // accumulate
  c->log.n = 0;
  (void)hipEventRecord(c->log.ev[0], c->stream);
  c->stats.gate_requests = 0;
  c->stats.gate_pending = 0;
  for (size_t k = 0; k < c->chunks.size(); k++) {
    const gi_ctx::Chunk& ch = c->chunks[k];
    if (B.gate && ch.n_body && c->prog.body_access) c->stats.gate_requests += ch.n_body;
    if (k && c->ctr.p) {
      e = hipMemsetAsync(c->ctr.p, 0, 128, c->stream);
      if (e != hipSuccess) return hip_fail(c, e, "memset chunk counters");
    }
    if (B.hdkeys) {  // the dedup table is per chunk (its entries name chunk-local requests)
      e = hipMemsetAsync(B.hdkeys, 0, 8ull * (c->hdmask + 1), c->stream);
      if (e == hipSuccess) e = hipMemsetAsync(B.hdinfo, 0, 8ull * (c->hdmask + 1), c->stream);
      if (e != hipSuccess) return hip_fail(c, e, "memset header dedup table");
    }
    DBatch Bc = B;
    Bc.n_req = ch.n;
    Bc.reqs = B.reqs + ch.r0;
    Bc.layout = B.layout + ch.r0;
    Bc.verdicts = B.verdicts + ch.r0;
    Bc.matched = B.matched + (uint64_t)ch.r0 * B.mcap;
    Bc.caprec = B.caprec ? B.caprec + 4ull * B.crcap * ch.r0 : nullptr;
    Bc.capbytes = B.capbytes ? B.capbytes + (uint64_t)B.cbcap * ch.r0 : nullptr;
    Bc.hits = B.hits + ch.r0;
    Bc.txslots = (Slot*)((uint8_t*)B.txslots + (uint64_t)GI_SLOT_BYTES * ch.r0);
    Bc.body_list = B.body_list + ch.blist_off;
    Bc.pend = B.pend ? B.pend + ch.r0 : nullptr;
    Bc.eorder = B.eorder ? B.eorder + ch.r0 : nullptr;
    Bc.eord_key = B.eord_key ? B.eord_key + ch.r0 : nullptr;
    Bc.n_body = ch.n_body;
    Bc.n_mp_body = ch.n_mp;
    launch_pipeline(c->prog, Bc, c->scan, c->stream, c->evs, c->stop_after, &c->log,
                    (const uint32_t*)c->tally_idbuf.p, (uint32_t)c->tally_ids.size());
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(c, e, "launch pipeline");
  (void)hipEventRecord(c->ev1, c->stream);
  c->ran = true;
  c->stats.batches++;
  return GI_OK;
}

int gi_sync(gi_ctx* c) {
  if (!c) return GI_EINVAL;
  (void)hipSetDevice(c->device);
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "stream sync");
  if (c->ran) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->stats.last_kernel_ms = ms;
    if (c->n_req && hipEventElapsedTime(&ms, c->ev0, c->evs[0]) == hipSuccess) c->stats.last_collect_ms = ms;
    if (c->n_req && hipEventElapsedTime(&ms, c->evs[0], c->evs[1]) == hipSuccess) c->stats.last_stream_ms = ms;
    if (c->n_req && hipEventElapsedTime(&ms, c->evs[1], c->evs[2]) == hipSuccess) c->stats.last_scan_ms = ms;
    if (c->n_req && hipEventElapsedTime(&ms, c->evs[2], c->ev1) == hipSuccess) c->stats.last_eval_ms = ms;
    // per-launch HIP-event times and algorithmic bytes
    uint64_t acct[16] = {0};
    if (c->ctr.p) (void)hipMemcpy(acct, (uint8_t*)c->ctr.p + 160, 128, hipMemcpyDeviceToHost);
    uint64_t acct2[6] = {0};
    if (c->ctr.p) (void)hipMemcpy(acct2, (uint8_t*)c->ctr.p + 336, 48, hipMemcpyDeviceToHost);
    uint32_t ibk[16] = {0};
    if (c->ctr.p) (void)hipMemcpy(ibk, (uint8_t*)c->ctr.p + 64, 64, hipMemcpyDeviceToHost);
    gi_tally tl{};
    (void)hipMemcpy(&tl, c->tally.p, sizeof(tl), hipMemcpyDeviceToHost);
    uint64_t ibc[5] = {0};  // items per bucket over all chunks (k_ioffsets)
    if (c->ctr.p) (void)hipMemcpy(ibc, (uint8_t*)c->ctr.p + 384, 40, hipMemcpyDeviceToHost);
    uint64_t slow_bytes = 0;
    if (c->ctr.p) (void)hipMemcpy(&slow_bytes, (uint8_t*)c->ctr.p + 8, 8, hipMemcpyDeviceToHost);
    uint32_t gate_pending = 0;  // DBatch.pcount[1] (kernels.hip eval_request)
    if (c->ctr.p) (void)hipMemcpy(&gate_pending, (uint8_t*)c->ctr.p + 516, 4, hipMemcpyDeviceToHost);
    c->stats.gate_pending = c->stats.gate_requests ? gate_pending : 0;
    if (c->gate_ran && c->stats.gate_requests)
      c->gate_pending_share = (double)c->stats.gate_pending / (double)c->stats.gate_requests;
    // one record per launch name: a chunked batch repeats the pipeline, its
    // launches of one name are summed
    uint32_t nrec = 0;
    for (int k = 0; k < c->log.n; k++) {
      float lm = 0;
      (void)hipEventElapsedTime(&lm, c->log.ev[k], c->log.ev[k + 1]);
      const std::string nm = c->log.name[k];
      uint32_t i = 0;
      while (i < nrec && nm != c->stats.launch_name[i]) i++;
      if (i == nrec) {
        if (nrec == GI_STATS_LAUNCHES) continue;
        nrec++;
        c->stats.launch_ms[i] = 0;
        snprintf(c->stats.launch_name[i], sizeof(c->stats.launch_name[i]), "%s", nm.c_str());
      }
      c->stats.launch_ms[i] += lm;
    }
    c->stats.n_launches = nrec;
    for (uint32_t k = 0; k < nrec; k++) {
      const std::string nm = c->stats.launch_name[k];
      uint64_t ab = 0;
      if (nm == "k_collect") ab = c->raw_nobody + (uint64_t)GI_REQHDR_BYTES * c->n_req;  // request bytes in, ReqHdr out
      else if (nm == "k_items") ab = 32ull * (ibc[0] + ibc[1] + ibc[2] + ibc[3] + ibc[4]);  // item records out
      else if (nm == "k_ioffsets") ab = 8ull * GI_NCLS * ((c->n_req + 255) / 256);       // block counts in, offsets out
      else if (nm.rfind("k_stream", 0) == 0) {
        const int b = nm.back() - '0';
        ab = acct[b] + 32ull * ibc[b] + 4ull * acct[5 + b];  // item bytes + records in, queue words out
      } else if (nm == "k_scan") ab = 4ull * acct[10];  // each stream's queue words once
      else if (nm == "k_scan_big") ab = 4ull * acct[11];
      else if (nm == "k_scan_hbm") ab = 4ull * acct[12];
      else if (nm == "k_scan_slow") ab = slow_bytes;
      else if (nm == "k_body") ab = c->raw_all - c->raw_nobody;  // request bodies
      else if (nm == "k_bparse" || nm == "k_mpparse") ab = c->raw_all - c->raw_nobody;
      else if (nm == "k_eval") ab = c->raw_all + (uint64_t)sizeof(gi_verdict) * c->n_req + 4ull * tl.matched_total;
      c->stats.launch_alg_bytes[k] = ab;
      c->stats.launch_steps[k] = nm == "k_scan" ? acct[13] : nm == "k_scan_big" ? acct[14] : nm == "k_scan_hbm" ? acct[15]
                                 : nm.rfind("k_stream", 0) == 0 ? acct2[nm.back() - '0']
                                 : nm == "k_detect" ? acct2[5] : 0;
    }
#ifdef GI_DEBUG
    if (c->ctr.p) {
      uint32_t dbg[4];
      if (hipMemcpy(dbg, (uint8_t*)c->ctr.p + 128, 16, hipMemcpyDeviceToHost) == hipSuccess && dbg[1])
        fprintf(stderr, "GI_DEBUG bounds: line %u count %u a=%u b=%u\n", dbg[0], dbg[1], dbg[2], dbg[3]);
    }
#endif
    if (c->prof_on && c->prof.p) {
      unsigned long long h[128];
      if (hipMemcpy(h, c->prof.p, 1024, hipMemcpyDeviceToHost) == hipSuccess && c->n_req) {
        for (int b = 0; b < 5; b++)
          fprintf(stderr, "GI_PROF k_stream bucket %d (sum over waves, Mcyc): item %.1f chain %.1f out %.1f loop %.1f total %.1f\n",
                  b, h[40 + 5 * b] / 1e6, h[41 + 5 * b] / 1e6, h[42 + 5 * b] / 1e6, h[43 + 5 * b] / 1e6,
                  h[44 + 5 * b] / 1e6);
        for (int b = 0; b < 5; b++)
          fprintf(stderr, "GI_PROF k_stream bucket %d: fm+ballot %.1f run_chain(lane max) %.1f slowcheck+collapse %.1f "
                  "stream_vals %.1f det_push %.1f\n", b, h[80 + 3 * b] / 1e6, h[81 + 3 * b] / 1e6, h[82 + 3 * b] / 1e6,
                  h[24 + 2 * b] / 1e6, h[25 + 2 * b] / 1e6);
        for (uint32_t k = 0; k < 16 && k < c->rs->prog.body_links.size(); k++) {
          const DRule& R = c->rs->prog.rules[c->rs->prog.body_links[k]];
          fprintf(stderr, "GI_PROF k_body link %u id %d chain %u op %d: transform %.1f Mcyc, operator %.1f Mcyc (sum)\n",
                  c->rs->prog.body_links[k], R.id, R.tchain_len, c->rs->prog.ops[R.op].kind, h[96 + 2 * k] / 1e6,
                  h[97 + 2 * k] / 1e6);
        }
        if (h[16])
          fprintf(stderr,
                  "GI_PROF wave_parse_json per body (%.0f bodies): total %.0f cyc, refills %.1f (%.0f cyc), members %.0f: "
                  "key %.0f, build+hash %.0f, value+add %.0f cyc per member\n",
                  (double)h[16], (double)h[9] / h[16], (double)h[11] / h[16], (double)h[10] / h[16],
                  (double)h[15] / h[16], (double)h[12] / std::max(1.0, (double)h[15]),
                  (double)h[13] / std::max(1.0, (double)h[15]), (double)h[14] / std::max(1.0, (double)h[15]));
        const double n = c->n_req;
        fprintf(stderr,
                "GI_PROF k_eval per request: init %.0f cyc, phase1 %.0f, phase2 %.0f, total %.0f; rule visits %.1f, "
                "evaluated %.1f, matched %.1f; eval_rule %.0f cyc, actions %.0f cyc\n",
                h[0] / n, h[1] / n, h[2] / n, h[3] / n, h[4] / n, h[5] / n, h[6] / n, h[7] / n, h[8] / n);
        fprintf(stderr,
                "GI_PROF k_eval_wave per request: fields filtered %.1f, survivors exact %.1f / evaluated %.1f; "
                "filter %.0f cyc, ordered tests %.0f cyc\n",
                h[17] / n, h[18] / n, h[19] / n, h[20] / n, h[21] / n);
        std::vector<unsigned long long> rc(3000);
        if (hipMemcpy(rc.data(), (uint8_t*)c->prof.p + 1024, 24000, hipMemcpyDeviceToHost) == hipSuccess) {
          std::vector<std::pair<unsigned long long, uint32_t>> v;
          for (uint32_t i = 0; i < 1000 && i < c->rs->prog.rules.size(); i++) v.push_back({rc[i], i});
          std::sort(v.rbegin(), v.rend());
          for (int k = 0; k < 40 && k < (int)v.size(); k++) {
            const DRule& R = c->rs->prog.rules[v[k].second];
            const double ent = (double)rc[1000 + v[k].second];
            fprintf(stderr, "  rule link %u id %d phase %d hit_slot %d op %d vars %u chain %u: %.0f cyc/req; "
                    "entered by %.1f%% of requests, %.0f cyc and %.2f operator runs per entry\n",
                    v[k].second, R.id, R.phase, R.hit_slot, R.op >= 0 ? c->rs->prog.ops[R.op].kind : -1,
                    R.var_count, R.tchain_len, v[k].first / n, 100.0 * ent / n, ent > 0 ? v[k].first / ent : 0.0,
                    ent > 0 ? rc[2000 + v[k].second] / ent : 0.0);
          }
        }
      }
    }
    if (c->diag_on && c->ctr.p) {  // pool words, slow bytes, slow entries, items per bucket
      uint64_t h[16];
      if (hipMemcpy(h, c->ctr.p, 128, hipMemcpyDeviceToHost) == hipSuccess) {
        const uint32_t* ib = (const uint32_t*)(h + 8);
        c->stats.diag[0] = h[0];
        c->stats.diag[1] = h[1];
        c->stats.diag[2] = h[2] & 0xFFFFFFFFull;
        for (int b = 0; b < 5; b++) c->stats.diag[3 + b] = ib[2 * b + 1];
        uint64_t vc[5] = {0, 0, 0, 0, 0};
        if (hipMemcpy(vc, (uint8_t*)c->ctr.p + 288, 40, hipMemcpyDeviceToHost) == hipSuccess)
          fprintf(stderr, "GI_DIAG phase-A void events: field %llu long %llu slow %llu qcap %llu pool %llu "
                  "(pool used %llu of %llu words, slow %llu of %u entries, %llu of %llu bytes)\n",
                  (unsigned long long)vc[0], (unsigned long long)vc[1], (unsigned long long)vc[2],
                  (unsigned long long)vc[3], (unsigned long long)vc[4], (unsigned long long)h[0],
                  (unsigned long long)c->pool_cap, (unsigned long long)(h[2] & 0xFFFFFFFFull), c->slow_cap,
                  (unsigned long long)h[1], (unsigned long long)c->slow_bytes_cap);
        if (c->det_cap)  // @detectSQLi/@detectXSS candidates listed by k_stream (k_detect entries)
          fprintf(stderr, "GI_DIAG detect entries %llu (cap %u), bytes %llu (cap %llu)\n",
                  (unsigned long long)(h[3] & 0xFFFFFFFFull), c->det_cap, (unsigned long long)h[4],
                  (unsigned long long)c->det_bytes_cap);
      }
    }
  }
  return GI_OK;
}

int gi_fetch_results(gi_ctx* c, gi_results* out) {
  if (!c || !out) return GI_EINVAL;
  if (!c->ran) return fail(c, GI_ESTATE, "gi_fetch_results before gi_run_staged");
  if (out->matched_cap != c->mcap) return fail(c, GI_ETRUNC, "matched_cap differs from the context's");
  int rc = gi_sync(c);
  if (rc != GI_OK) return rc;
  hipError_t e = hipSuccess;
  if (c->n_req && out->verdicts)
    e = hipMemcpy(out->verdicts, c->verdicts.p, (size_t)c->n_req * sizeof(gi_verdict), hipMemcpyDeviceToHost);
  if (e == hipSuccess && c->n_req && out->matched_ids)
    e = hipMemcpy(out->matched_ids, c->matched.p, (size_t)c->n_req * c->mcap * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && c->n_req && (out->captures || out->capture_bytes)) {
    if (out->capture_cap != c->staged_crcap || out->capture_bytes_cap != c->staged_cbcap)
      return fail(c, GI_ETRUNC, "capture caps differ from the context's");
    if (!c->cap_on) {  // no observable capture in the ruleset: empty rows
      if (out->captures) memset(out->captures, 0, sizeof(gi_capture) * c->n_req * c->staged_crcap);
    } else {
      if (out->captures)
        e = hipMemcpy(out->captures, c->caprec.p, sizeof(gi_capture) * c->n_req * c->staged_crcap, hipMemcpyDeviceToHost);
      if (e == hipSuccess && out->capture_bytes)
        e = hipMemcpy(out->capture_bytes, c->capbytes.p, (size_t)c->n_req * c->staged_cbcap, hipMemcpyDeviceToHost);
    }
  }
  if (e != hipSuccess) return hip_fail(c, e, "fetch D2H");
  return GI_OK;
}

int gi_tally_get(gi_ctx* c, gi_tally* out) {
  if (!c || !out) return GI_EINVAL;
  if (!c->ran) return fail(c, GI_ESTATE, "no batch has run");
  int rc = gi_sync(c);
  if (rc != GI_OK) return rc;
  hipError_t e = hipMemcpy(out, c->tally.p, sizeof(gi_tally), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(c, e, "fetch tally");
  return GI_OK;
}

int gi_tally_detail_get(gi_ctx* c, uint64_t* score_hist, uint32_t* rule_ids, uint64_t* rule_hits, uint32_t cap,
                        uint32_t* n_rules) {
  if (!c) return GI_EINVAL;
  const uint32_t nt = (uint32_t)c->tally_ids.size();
  if (n_rules) *n_rules = nt;
  if (!score_hist && !rule_ids && !rule_hits) return GI_OK;  // size query
  if (!c->ran) return fail(c, GI_ESTATE, "no batch has run");
  if ((rule_ids || rule_hits) && cap < nt) return fail(c, GI_ETRUNC, "rule tally capacity too small");
  int rc = gi_sync(c);
  if (rc != GI_OK) return rc;
  std::vector<uint32_t> h(GI_SCORE_BINS + nt);
  hipError_t e = hipMemcpy(h.data(), c->tally_ext.p, 4 * h.size(), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(c, e, "fetch detail tally");
  if (score_hist)
    for (int b = 0; b < GI_SCORE_BINS; b++) score_hist[b] = h[b];
  for (uint32_t k = 0; k < nt; k++) {
    if (rule_ids) rule_ids[k] = c->tally_ids[k];
    if (rule_hits) rule_hits[k] = h[GI_SCORE_BINS + k];
  }
  return GI_OK;
}

int gi_stats_get(gi_ctx* c, gi_stats* out) {
  if (!c || !out) return GI_EINVAL;
  *out = c->stats;
  return GI_OK;
}

// CPU baseline (Coraza Go is absent here, so "the build's own
// C++ CPU restatement, multi-threaded on all cores and labelled as such"):
// the interpreter k_collect / k_eval run, compiled for the host
// (kernels.hip cpu_inspect_one), one request at a time per thread, with no
// phase A (every rule link evaluated by the interpreter).  Not a fallback of
// the inspection path: gi_inspect_* never calls it.
int gi_cpu_baseline_inspect(const gi_ruleset* rs, const gi_batch* in, gi_results* out, uint32_t n_threads,
                            double* eval_seconds) {
  if (!rs || !in || !out || !out->verdicts || !out->matched_ids || out->matched_cap == 0) return GI_EINVAL;
  if (in->n_req && (!in->reqs || !in->data)) return GI_EINVAL;
  try {
    const Program& PG = rs->prog;
    std::vector<std::vector<uint8_t>> store;
    auto put = [&](const void* src, size_t bytes) -> const void* {
      store.emplace_back(bytes + 64, 0);
      if (bytes) memcpy(store.back().data(), src, bytes);
      return store.back().data();
    };
    DProgram np{};
    std::vector<uint32_t> top_ph;
    uint32_t n_ph1 = 0;
    if (const char* ferr = fill_dprogram(PG, np, put, top_ph, n_ph1)) {
      (void)ferr;
      return GI_EINVAL;
    }
    // the interpreter's word readers may look up to 7 bytes past a value: a padded arena
    std::vector<uint8_t> data(in->data_len + 64, 0);
    if (in->data_len) memcpy(data.data(), in->data, in->data_len);
    const uint32_t n = in->n_req;
    const uint32_t nt = std::max(1u, std::min<uint32_t>(n_threads ? n_threads : std::thread::hardware_concurrency(),
                                                        std::max(1u, n)));
    std::atomic<uint32_t> next(0);
    std::atomic<int> bad(GI_OK);
    const bool layout_debug = getenv("GI_LAYOUT_DEBUG") != nullptr;  // read once, before the threads
    auto work = [&]() {
      std::vector<uint64_t> scratch, capture;
      std::vector<uint64_t> txs(2ull * std::max<uint32_t>(PG.n_slots, 1));
      for (;;) {
        const uint32_t lo = next.fetch_add(64);
        if (lo >= n || bad.load() != GI_OK) return;
        for (uint32_t r = lo; r < std::min(n, lo + 64); r++) {
          ReqLayout L{};
          LayoutSizes z{};
          LayoutAcc acc;
          if (const char* lerr = request_layout(PG, np.cap_ws_words, np.cap_groups, in, r, L, z, acc)) {
            if (strncmp(lerr, "request too large", 17) != 0) {  // malformed input: the call fails
              bad.store(GI_EINVAL);
              return;
            }
            // a request beyond the per-request capacities: flagged, like the GPU path does
            gi_verdict& v = out->verdicts[r];
            memset(&v, 0, sizeof(v));
            v.flags = GI_REQ_OVERFLOW;
            continue;
          }
          L.base = 0;
          L.vmap_bit = 0;
          L.hset_word = 0;
          L.hset_mask = 0;  // no phase A: no hit set
          L.cap_off = 0;
          if (layout_debug && z.region > (1u << 20))  // diagnostics: what sizes a large region
            fprintf(stderr, "GI_LAYOUT r=%u region=%llu cap_f=%u cap_b=%u cap_t=%u cap_mt=%u dyn=%u/%u mv=%u/%u capb=%llu\n", r,
                    (unsigned long long)z.region, L.cap_f, L.cap_b, L.cap_t, L.cap_mt, L.dyn_cap, L.dyn_capb, L.mv_cap_e,
                    L.mv_cap_a, (unsigned long long)z.capb);
          const size_t words = (z.region + 64) / 8 + 8;
          if (scratch.size() < words) scratch.assign(words, 0);
          const size_t cwords = (z.capb + 64) / 8 + 8;
          if (capture.size() < cwords) capture.assign(cwords, 0);
          DBatch B{};
          B.data = data.data();
          B.reqs = in->reqs + r;
          B.headers = in->headers;
          B.n_req = 1;
          B.rstride = 1;
          B.mcap = out->matched_cap;
          B.scratch = (uint8_t*)scratch.data();
          B.cappool = (uint8_t*)capture.data();
          B.prog = &np;
          B.layout = &L;
          B.verdicts = out->verdicts + r;
          B.matched = out->matched_ids + (uint64_t)r * out->matched_cap;
          if (out->captures && out->capture_bytes && out->capture_cap) {  // capture records, as gi_fetch_results
            B.caprec = (uint32_t*)(out->captures + (uint64_t)r * out->capture_cap);
            B.capbytes = out->capture_bytes + (uint64_t)r * out->capture_bytes_cap;
            B.crcap = out->capture_cap;
            B.cbcap = out->capture_bytes_cap;
          }
          B.txslots = (Slot*)txs.data();
          cpu_inspect_one(np, B);
        }
      }
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (uint32_t k = 1; k < nt; k++) {
      try {
        th.emplace_back(work);
      } catch (...) {
        break;  // run with the threads the system gave us
      }
    }
    work();
    for (auto& x : th) x.join();
    if (eval_seconds)
      *eval_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return bad.load();
  } catch (const std::bad_alloc&) {
    return GI_ENOMEM;
  } catch (...) {
    return GI_EINVAL;
  }
}

int gi_inspect_batch(gi_ctx* c, const gi_batch* in, gi_results* out) {
  int rc = gi_stage_batch(c, in);
  if (rc != GI_OK) return rc;
  rc = gi_run_staged(c);
  if (rc != GI_OK) return rc;
  return gi_fetch_results(c, out);
}

int gi_selftest_regex_many(const char* pattern, size_t plen, const uint8_t* data, const uint64_t* offs, uint32_t n,
                           uint8_t* out, uint32_t* n_states) {
  if (!pattern || (n && (!data || !offs || !out))) return GI_EINVAL;
  Regex re;
  std::string err;
  if (!re_parse(std::string(pattern, plen), &re, &err)) return GI_EPARSE;
  Dfa d;
  NfaTables t;
  const bool dfa = build_regex_dfa(re, &d, &err);
  if (!dfa && !build_nfa_tables(re, &t, &err)) return GI_EUNSUPPORTED;
  if (n_states) *n_states = dfa ? d.n_states : 0;
  for (uint32_t k = 0; k < n; k++) {
    const uint8_t* s = data + offs[k];
    const size_t len = offs[k + 1] - offs[k];
    out[k] = (dfa ? dfa_host_match(d, s, len) : nfa_host_match(t, s, len)) ? 1 : 0;
  }
  return GI_OK;
}

int gi_selftest_capture(const char* pattern, size_t plen, const uint8_t* s, size_t n, int32_t* caps,
                        uint32_t* nslot) {
  if (!pattern || (n && !s) || !caps || !nslot) return GI_EINVAL;
  Regex re;
  std::string err;
  if (!re_parse("(?sm)" + std::string(pattern, plen), &re, &err)) return GI_EPARSE;
  std::vector<DPikeInst> insts;
  std::vector<uint32_t> pool;
  DPike pk{};
  if (!build_pike(re, &insts, &pool, &pk, &err)) return GI_EUNSUPPORTED;
  std::vector<uint32_t> ws(pike_ws_words(pk.n_inst, pk.nslot));
  *nslot = pk.nslot;
  return pike_match(insts.data() + pk.inst_off, pool.data(), pk, s, (uint32_t)n, ws.data(), caps) ? 1 : 0;
}

int gi_selftest_regex(const char* pattern, size_t plen, const uint8_t* s, size_t n, uint32_t* n_states) {
  Regex re;
  std::string err;
  if (!re_parse(std::string(pattern, plen), &re, &err)) return GI_EPARSE;
  Dfa d;
  if (!build_regex_dfa(re, &d, &err)) {  // the compiler's fallback: exact NFA tables
    NfaTables t;
    if (!build_nfa_tables(re, &t, &err)) return GI_EUNSUPPORTED;
    if (n_states) *n_states = 0;
    return nfa_host_match(t, s, n) ? 1 : 0;
  }
  if (n_states) *n_states = d.n_states;
  return dfa_host_match(d, s, n) ? 1 : 0;
}

}  // extern "C"

// ------------------------------------------------------------ plan self-test
// Host emulation of k_scan over every job image (compiler self-test only; the
// inspection path never runs on the host): structural bounds of each image
// and, on pseudo-random ASCII inputs, the image walk (joint class map, u16
// transitions, end-of-input tables, slot table) against the global tables
// the per-value path uses.  Returns 0 or the number of the first failed check.
namespace {
uint64_t host_scan_global(const Program& P, const DDfa& d, const uint8_t* s, size_t n) {
  const uint16_t* tr = &P.trans[d.trans_off];
  const uint8_t* amap = &P.u8pool[d.amap_off];
  uint32_t st = d.start;
  uint64_t m = 0;
  for (size_t i = 0; i < n; i++) {
    if (!d.multi && st == d.accept) return 1;
    const uint32_t cls = amap[s[i]];
    const uint32_t tv = tr[(size_t)st * d.n_classes + cls];
    if (d.multi) {
      if (tv & 0x8000) m |= P.u64pool[d.acc_off + (size_t)st * 5 + P.u8pool[d.combo_off + cls]];
      st = tv & 0x7FFF;
    } else {
      st = tv;
    }
  }
  if (d.multi) return m | P.u64pool[d.acc_off + (size_t)st * 5 + 4];
  return P.u8pool[d.endacc_off + st] ? 1 : 0;
}
}  // namespace

extern "C" int gi_selftest_plan(const gi_ruleset* rs, char* err, size_t errcap) {
  if (!rs) return GI_EINVAL;
  const Program& P = rs->prog;
  auto bad = [&](int code, const std::string& m) {
    if (err && errcap) snprintf(err, errcap, "%s", m.c_str());
    return code;
  };
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  for (size_t j = 0; j < P.jobs.size(); j++) {
    const DJob& J = P.jobs[j];
    if (J.stream >= P.streams.size()) return bad(1, "job stream");
    if ((uint64_t)J.img_off + J.img_bytes > P.images.size()) return bad(2, "image range");
    if (J.jdfa_count == 0 || J.jdfa_count > GI_JOB_MAX_DFA) return bad(3, "automata per job");
    const uint8_t* img = &P.images[J.img_off];
    const uint32_t nf = (uint32_t)P.filters.size();
    if ((uint64_t)J.lds_fmask + 8ull * J.jdfa_count * nf > J.img_bytes) return bad(4, "fmask table");
    if (J.lds && (J.big ? J.img_bytes > GI_BIG_LDS_BYTES + 4096 : J.img_bytes > GI_JOB_LDS_BYTES))
      return bad(5, "lds image size");
    for (uint32_t q = 0; q < J.jdfa_count; q++) {
      const DJobDfa& jd = P.jdfas[J.jdfa_begin + q];
      const DDfa& d = P.dfas[jd.dfa];
      const uint64_t tb = 2ull * d.n_states * d.n_classes;
      if (jd.lds_trans < 0 || (uint64_t)jd.lds_trans + tb > J.img_bytes) return bad(6, "transitions");
      if (jd.lds_amap < 0 || (uint64_t)jd.lds_amap + 128 > J.img_bytes) return bad(7, "class map");
      if (jd.lds_endacc < 0 || (uint64_t)jd.lds_endacc + (d.multi ? 8ull : 1ull) * d.n_states > J.img_bytes)
        return bad(8, "end accept");
      if (jd.lds_slots < 0 || (uint64_t)jd.lds_slots + 4ull * jd.n_pat > J.img_bytes) return bad(9, "slots");
      if (d.multi && (jd.lds_combo < 0 || (uint64_t)jd.lds_combo + d.n_classes > J.img_bytes)) return bad(10, "combo");
      if (d.start >= d.n_states) return bad(11, "start state");
      const uint16_t* tr = (const uint16_t*)(img + jd.lds_trans);
      for (uint64_t k = 0; k < (uint64_t)d.n_states * d.n_classes; k++) {
        const uint32_t nx = d.multi ? (tr[k] & 0x7FFFu) : tr[k];
        if (nx >= d.n_states) return bad(12, "transition target");
      }
      for (uint32_t c = 0; c < 128; c++) {
        const uint32_t jc = (((const uint32_t*)img)[c] >> (8 * q)) & 0xFF;
        if (jc >= d.n_classes || jc != img[jd.lds_amap + c]) return bad(13, "joint class map");
      }
      if (P.streams[J.stream].collapse) {  // every rune-mapped byte lands in the automaton's class of its runes
        const DStream& S = P.streams[J.stream];
        if (d.byte_mode) return bad(20, "rune-mapped stream with a byte-mode automaton");
        auto cls_of = [&](uint32_t r) -> uint32_t {
          for (uint32_t k = 0; k < d.nr_cnt; k++)
            if (P.nranges[d.nr_off + 3 * k] <= r && r <= P.nranges[d.nr_off + 3 * k + 1]) return P.nranges[d.nr_off + 3 * k + 2];
          return 0;
        };
        if (S.rmap_cnt == 0) {
          if (!d.nonascii_uniform || ((((const uint32_t*)img)[128] >> (8 * q)) & 0xFF) != d.nonascii_cls)
            return bad(20, "collapsed stream with a rune-distinguishing automaton");
        }
        for (uint32_t k = 0; k < S.rmap_cnt; k++) {
          const uint32_t lo = P.nranges[S.rmap_off + 3 * k], hi = P.nranges[S.rmap_off + 3 * k + 1];
          const uint32_t b = P.nranges[S.rmap_off + 3 * k + 2];
          const uint32_t jc = (((const uint32_t*)img)[b] >> (8 * q)) & 0xFF;
          if (jc != cls_of(lo) || jc != cls_of(hi) || jc != cls_of(lo + (hi - lo) / 2))
            return bad(22, "rune map byte in another class than its runes");
        }
      }
      for (uint32_t k = 0; k < jd.n_pat; k++)
        if (*(const uint32_t*)(img + jd.lds_slots + 4 * k) != P.pats[jd.pat_begin + k].slot) return bad(14, "slot table");
      // image walk == global-table walk on random ASCII strings
      uint8_t s[96];
      for (int trial = 0; trial < 64; trial++) {
        const size_t n = rnd() % sizeof(s);
        for (size_t i = 0; i < n; i++) s[i] = (uint8_t)(32 + rnd() % 95);
        uint32_t st = d.start;
        uint64_t m = 0;
        for (size_t i = 0; i < n; i++) {
          const uint32_t cls = (((const uint32_t*)img)[s[i] & 0x7F] >> (8 * q)) & 0xFF;
          const uint32_t tv = tr[(size_t)st * d.n_classes + cls];
          if (d.multi) {
            if (tv & 0x8000) m |= P.u64pool[d.acc_off + (size_t)st * 5 + img[jd.lds_combo + cls]];
            st = tv & 0x7FFF;
          } else {
            st = tv;
          }
        }
        const uint64_t bits = d.multi ? (m | *(const uint64_t*)(img + jd.lds_endacc + 8 * st))
                                      : (img[jd.lds_endacc + st] ? 1ull : 0ull);
        if (bits != host_scan_global(P, d, s, n)) return bad(15, "image walk differs from the global tables");
      }
    }
  }
  for (size_t s = 0; s < P.streams.size(); s++) {
    const DStream& S = P.streams[s];
    if ((uint64_t)S.filt_begin + S.filt_count > P.sfilt.size()) return bad(16, "stream filters");
    uint64_t gm = 0;
    for (uint32_t k = 0; k < S.filt_count; k++) {
      if (P.sfilt[S.filt_begin + k] >= P.filters.size()) return bad(17, "global filter id");
      gm |= 1ull << P.sfilt[S.filt_begin + k];
    }
    if (gm != S.gmask) return bad(21, "stream filter mask");
    if ((uint64_t)S.job_begin + S.job_count > P.jobs.size()) return bad(18, "stream jobs");
    for (uint32_t j = S.job_begin; j < S.job_begin + S.job_count; j++)
      if (P.jobs[j].stream != s) return bad(19, "job/stream mismatch");
  }
  return 0;
}

// Transformation identity triggers (compiler/kernel self-test): triggers[code]
// for code < n_codes and the byte summary of every byte value.
extern "C" int gi_selftest_triggers(uint32_t* triggers, uint32_t n_codes, uint32_t* byte_summaries) {
  if (!triggers || !byte_summaries) return GI_EINVAL;
  for (uint32_t c = 0; c < n_codes; c++) triggers[c] = transform_triggers((uint8_t)c);
  for (uint32_t b = 0; b < 256; b++) byte_summaries[b] = byte_summary((uint8_t)b);
  return GI_OK;
}
