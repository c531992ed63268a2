// Host runtime of the C ABI (include/gpuinspect.h): compile, device context,
// batch staging (H2D + per-request scratch layout), launch, result fetch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpuinspect.h"
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
    "anomaly_score", "0"};

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
  DevBuf data, reqs, hdrs, layout, scratch, verdicts, matched, tally, hits, tscratch;
  uint32_t scan_threads = 0;
  uint32_t tcap = 2048;
  uint32_t hit_words = 0;
  hipEvent_t evs[2] = {nullptr, nullptr};
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
  int rc = compile_program(std::string(seclang, n), exports, opts ? opts->dfa_state_cap : 0, &rs->prog, &msg);
  if (rc != 0) {
    if (err && errcap) {
      size_t k = std::min(errcap - 1, msg.size());
      memcpy(err, msg.data(), k);
      err[k] = 0;
    }
    delete rs;
    return rc == -1 ? GI_EPARSE : GI_EUNSUPPORTED;
  }
  const Program& P = rs->prog;
  rs->info.n_rules = (uint32_t)P.top.size();
  rs->info.n_links = (uint32_t)P.rules.size();
  rs->info.n_dfas = (uint32_t)P.dfas.size();
  rs->info.n_tx_slots = P.n_slots;
  rs->info.n_scan_jobs = (uint32_t)P.jobs.size();
  rs->info.n_scan_streams = (uint32_t)P.streams.size();
  rs->info.n_hit_slots = P.n_hit_slots;
  rs->info.n_union_dfas = P.n_union_dfas;
  rs->info.program_bytes = P.rules.size() * sizeof(DRule) + P.vars.size() * sizeof(DVarRef) +
                           P.ops.size() * sizeof(DOp) + P.acts.size() * sizeof(DAction) +
                           P.trans.size() * 2 + P.u8pool.size() + P.nranges.size() * 4 + P.strpool.size() +
                           P.dfas.size() * sizeof(DDfa) + P.tparts.size() * sizeof(DTmplPart) +
                           P.u64pool.size() * 8 + P.streams.size() * sizeof(DStream) +
                           P.filters.size() * sizeof(DFilter) + P.jobs.size() * sizeof(DJob) +
                           P.jdfas.size() * sizeof(DJobDfa) + P.pats.size() * sizeof(DPat) +
                           P.svals.size() * sizeof(DScanVal) + P.images.size();
  *out = rs;
  return GI_OK;
}

void gi_ruleset_free(gi_ruleset* rs) { delete rs; }

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

int gi_ctx_create(const gi_ruleset* rs, int device, uint32_t matched_cap, gi_ctx** out) {
  if (!rs || !out) return GI_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return GI_ENODEV;
  auto* c = new gi_ctx();
  c->rs = rs;
  c->device = device;
  c->mcap = matched_cap ? matched_cap : 64;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e == hipSuccess) e = hipEventCreate(&c->evs[0]);
  if (e == hipSuccess) e = hipEventCreate(&c->evs[1]);
  if (e != hipSuccess) {
    delete c;
    return GI_ENODEV;
  }
  const Program& P = rs->prog;
  c->pbufs.resize(32);
  std::vector<uint32_t> lower;
  lower.reserve(GI_N_LOWER_PAIRS * 2);
  for (int i = 0; i < GI_N_LOWER_PAIRS; i++) {
    lower.push_back(kLowerPairs[i][0]);
    lower.push_back(kLowerPairs[i][1]);
  }
  hipStream_t s = c->stream;
  int k = 0;
  e = hipSuccess;
#define UP(field, vec, T)                                   \
  if (e == hipSuccess) {                                    \
    e = upload(&c->pbufs[k], vec, s);                       \
    c->prog.field = (const T*)c->pbufs[k].p;                \
    k++;                                                    \
  }
  UP(rules, P.rules, DRule)
  UP(top, P.top, uint32_t)
  UP(vars, P.vars, DVarRef)
  UP(excs, P.excs, DExc)
  UP(ops, P.ops, DOp)
  UP(acts, P.acts, DAction)
  UP(tparts, P.tparts, DTmplPart)
  UP(tmpls, P.tmpls, DTmpl)
  UP(tchains, P.tchains, uint8_t)
  UP(dfas, P.dfas, DDfa)
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
#undef UP
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    gi_ctx_free(c);
    return GI_ENODEV;
  }
  c->prog.n_lower_pairs = GI_N_LOWER_PAIRS;
  c->prog.n_top = (uint32_t)P.top.size();
  c->prog.n_slots = P.n_slots;
  c->prog.n_markers = P.n_markers;
  c->prog.n_exports = (uint32_t)P.exports.size();
  for (int i = 0; i < 8; i++) c->prog.exports[i] = i < (int)P.exports.size() ? P.exports[i] : -1;
  c->prog.rule_engine = P.rule_engine;
  c->prog.body_access = P.body_access;
  c->prog.body_limit = P.body_limit;
  c->prog.n_jobs = (uint32_t)P.jobs.size();
  c->prog.max_img_bytes = P.max_img_bytes;
  c->prog.n_hit_slots = P.n_hit_slots;
  c->scan_threads = scan_resident_threads(P.max_img_bytes);
  if (c->tscratch.ensure((size_t)c->scan_threads * 2 * c->tcap) != hipSuccess) {
    gi_ctx_free(c);
    return GI_ENOMEM;
  }
  *out = c;
  return GI_OK;
}

void gi_ctx_free(gi_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& b : c->pbufs) b.release();
  for (DevBuf* b : {&c->data, &c->reqs, &c->hdrs, &c->layout, &c->scratch, &c->verdicts, &c->matched, &c->tally,
                    &c->hits, &c->tscratch})
    b->release();
  for (auto& ev : c->evs)
    if (ev) (void)hipEventDestroy(ev);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* gi_last_error(const gi_ctx* c) { return c ? c->err.c_str() : "null context"; }

void* gi_ctx_stream(gi_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gi_stage_batch(gi_ctx* c, const gi_batch* in) {
  if (!c || !in) return GI_EINVAL;
  if (in->n_req && (!in->reqs || !in->data)) return fail(c, GI_EINVAL, "null batch arrays");
  (void)hipSetDevice(c->device);
  auto t0 = std::chrono::steady_clock::now();
  const uint32_t n = in->n_req;
  // validate spans and lay out per-request scratch (lengths only)
  std::vector<ReqLayout> lay(n);
  uint64_t off = 0;
  const uint32_t nslots = c->rs->prog.n_slots;
  for (uint32_t r = 0; r < n; r++) {
    const gi_request& q = in->reqs[r];
    const gi_span* sp[4] = {&q.method, &q.uri, &q.proto, &q.body};
    for (auto* s : sp)
      if (s->off + s->len > in->data_len) return fail(c, GI_EINVAL, "request span out of range");
    if ((uint64_t)q.hdr_begin + q.hdr_count > in->n_headers) return fail(c, GI_EINVAL, "header range out of range");
    uint64_t maxv = std::max<uint64_t>({(uint64_t)q.uri.len * 3 + 2, (uint64_t)q.method.len + q.uri.len + q.proto.len + 2,
                                        (uint64_t)q.body.len, 64});
    uint64_t cookie = 0, ncookie = 0;
    for (uint32_t h = 0; h < q.hdr_count; h++) {
      const gi_header& hd = in->headers[q.hdr_begin + h];
      if (hd.name.off + hd.name.len > in->data_len || hd.value.off + hd.value.len > in->data_len)
        return fail(c, GI_EINVAL, "header span out of range");
      maxv = std::max<uint64_t>(maxv, std::max(hd.name.len, hd.value.len));
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
    uint64_t cap_f = q.hdr_count + (q.uri.len / 2 + 2) + (cookie / 2 + 2 * ncookie) + (q.body.len / 2 + 2);
    uint64_t cap_b = 4ull * q.uri.len + q.method.len + q.proto.len + q.body.len + 96;
    uint64_t cap_t = 3 * maxv + 64;
    uint64_t cap_mt = 2 * maxv + 512;
    if (cap_f > 0xFFFFFFFFull || cap_b > 0xFFFFFFFFull || cap_t > 0xFFFFFFFFull || cap_mt > 0xFFFFFFFFull)
      return fail(c, GI_EINVAL, "request too large");
    ReqLayout& L = lay[r];
    L.base = off;
    L.cap_f = (uint32_t)cap_f;
    L.cap_b = (uint32_t)cap_b;
    L.cap_t = (uint32_t)cap_t;
    L.cap_mt = (uint32_t)cap_mt;
    uint64_t sz = 256 + cap_f * 32 + ((uint64_t)nslots * 24 + 15) / 16 * 16 + (cap_b + 15) / 16 * 16 +
                  2 * ((cap_t + 15) / 16 * 16) + 2 * ((cap_mt + 15) / 16 * 16);
    off += (sz + 63) / 64 * 64;
  }
  hipError_t e = hipSuccess;
  hipStream_t s = c->stream;
  if ((e = c->data.ensure(std::max<uint64_t>(in->data_len, 16))) != hipSuccess) return hip_fail(c, e, "alloc data");
  if ((e = c->reqs.ensure(std::max<size_t>(n * sizeof(gi_request), 16))) != hipSuccess) return hip_fail(c, e, "alloc reqs");
  if ((e = c->hdrs.ensure(std::max<size_t>(in->n_headers * sizeof(gi_header), 16))) != hipSuccess)
    return hip_fail(c, e, "alloc headers");
  if ((e = c->layout.ensure(std::max<size_t>(n * sizeof(ReqLayout), 16))) != hipSuccess) return hip_fail(c, e, "alloc layout");
  if ((e = c->scratch.ensure(std::max<uint64_t>(off, 64))) != hipSuccess) return hip_fail(c, e, "alloc scratch");
  if ((e = c->verdicts.ensure(std::max<size_t>(n * sizeof(gi_verdict), 16))) != hipSuccess)
    return hip_fail(c, e, "alloc verdicts");
  if ((e = c->matched.ensure(std::max<size_t>((size_t)n * c->mcap * 4, 16))) != hipSuccess)
    return hip_fail(c, e, "alloc matched");
  if ((e = c->tally.ensure(sizeof(gi_tally))) != hipSuccess) return hip_fail(c, e, "alloc tally");
  c->hit_words = (c->rs->prog.n_hit_slots + 31) / 32;
  if ((e = c->hits.ensure(std::max<size_t>((size_t)c->hit_words * n * 4, 16))) != hipSuccess)
    return hip_fail(c, e, "alloc hits");
  if (in->data_len) e = hipMemcpyAsync(c->data.p, in->data, in->data_len, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(c->reqs.p, in->reqs, n * sizeof(gi_request), hipMemcpyHostToDevice, s);
  if (e == hipSuccess && in->n_headers)
    e = hipMemcpyAsync(c->hdrs.p, in->headers, in->n_headers * sizeof(gi_header), hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n) e = hipMemcpyAsync(c->layout.p, lay.data(), n * sizeof(ReqLayout), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "stage H2D");
  c->n_req = n;
  c->staged = true;
  c->ran = false;
  c->stats.last_scratch_bytes = off;
  c->stats.last_stage_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GI_OK;
}

int gi_run_staged(gi_ctx* c) {
  if (!c) return GI_EINVAL;
  if (!c->staged) return fail(c, GI_ESTATE, "gi_run_staged before gi_stage_batch");
  (void)hipSetDevice(c->device);
  hipError_t e = hipMemsetAsync(c->tally.p, 0, sizeof(gi_tally), c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "memset tally");
  DBatch B;
  B.data = (const uint8_t*)c->data.p;
  B.reqs = (const gi_request*)c->reqs.p;
  B.headers = (const gi_header*)c->hdrs.p;
  B.n_req = c->n_req;
  B.mcap = c->mcap;
  B.scratch = (uint8_t*)c->scratch.p;
  B.layout = (const ReqLayout*)c->layout.p;
  B.verdicts = (gi_verdict*)c->verdicts.p;
  B.matched = (uint32_t*)c->matched.p;
  B.tally = (unsigned long long*)c->tally.p;
  B.hits = (uint32_t*)c->hits.p;
  B.tscratch = (uint8_t*)c->tscratch.p;
  B.tcap = c->tcap;
  (void)hipEventRecord(c->ev0, c->stream);
  if (c->hit_words) {
    e = hipMemsetAsync(c->hits.p, 0, (size_t)c->hit_words * c->n_req * 4, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "memset hits");
  }
  launch_pipeline(c->prog, B, c->scan_threads, c->stream, c->evs);
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
    if (c->n_req && hipEventElapsedTime(&ms, c->evs[0], c->evs[1]) == hipSuccess) c->stats.last_scan_ms = ms;
    if (c->n_req && hipEventElapsedTime(&ms, c->evs[1], c->ev1) == hipSuccess) c->stats.last_eval_ms = ms;
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

int gi_stats_get(gi_ctx* c, gi_stats* out) {
  if (!c || !out) return GI_EINVAL;
  *out = c->stats;
  return GI_OK;
}

int gi_inspect_batch(gi_ctx* c, const gi_batch* in, gi_results* out) {
  int rc = gi_stage_batch(c, in);
  if (rc != GI_OK) return rc;
  rc = gi_run_staged(c);
  if (rc != GI_OK) return rc;
  return gi_fetch_results(c, out);
}

int gi_selftest_regex(const char* pattern, size_t plen, const uint8_t* s, size_t n, uint32_t* n_states) {
  Regex re;
  std::string err;
  if (!re_parse(std::string(pattern, plen), &re, &err)) return GI_EPARSE;
  Dfa d;
  if (!build_regex_dfa(re, &d, &err)) return GI_EUNSUPPORTED;
  if (n_states) *n_states = d.n_states;
  return dfa_host_match(d, s, n) ? 1 : 0;
}

}  // extern "C"
