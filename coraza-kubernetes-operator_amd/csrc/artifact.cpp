// GPU artifact (de)serialisation.  Layout (little-endian):
//
//   header  : magic "GIARTFCT", u32 version, u32 n_sections, u64 payload bytes,
//             u64 FNV-1a 64 of the payload, u64 sizeof-signature of the records
//   payload : n_sections x { u32 tag, u32 elem_size, u64 count, bytes, pad to 8 }
//
// Every std::vector member of Program is one section of plain records; the
// scalars are one section; strings are byte sections.  The sizeof-signature
// and the per-section elem_size reject an artifact written by a build with a
// different record layout; the checksum rejects corruption.  See artifact.h.
#include "artifact.h"

#include <string.h>

#include <algorithm>

#include "../../include/gpuinspect.h"

namespace gi {

uint64_t fnv64(const uint8_t* p, size_t n, uint64_t h) {
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

namespace {

const char kMagic[8] = {'G', 'I', 'A', 'R', 'T', 'F', 'C', 'T'};

struct Scalars {
  uint8_t item_sides[8];
  uint32_t item_singles, n_hit_slots, n_union_dfas, max_img_bytes, max_big_img_bytes, n_slots, n_markers;
  uint8_t rule_engine, body_access, mv_used, body_partial, fold_on, _pad[3];
  uint32_t fold_nids, max_tx_lit;
  uint32_t n_rm_groups, args_limit;
  uint64_t body_limit, source_digest;
  uint64_t compiler_rev;  // fnv64 of kCompilerRev
};

uint64_t compiler_rev_hash() { return fnv64((const uint8_t*)kCompilerRev, strlen(kCompilerRev)); }

// One entry per Program vector: tag, member.  Order = file order.
#define GI_ART_VECTORS(X)                                                                                     \
  X(1, rules) X(2, top) X(3, vars) X(4, excs) X(5, ops) X(6, acts) X(7, tparts) X(8, tmpls) X(9, tchains)    \
  X(10, dfas) X(11, trans) X(12, u8pool) X(13, nranges) X(14, strpool) X(15, slot_names) X(16, u64pool)     \
  X(17, streams) X(18, filters) X(19, sfilt) X(20, body_links) X(21, always_slots) X(22, jobs) X(23, jdfas) \
  X(24, pats) X(25, svals) X(26, images) X(27, exports) X(28, nfas) X(29, pikes) X(30, pike_insts)              \
  X(31, pike_ranges) X(32, dyn_sites) X(33, txrx) X(34, tx_snap) X(35, fold_ids) X(36, fold_runs) \
  X(37, rule_groups)

constexpr uint32_t kTagScalars = 100, kTagPlan = 101, kTagExportNames = 102;

uint64_t layout_signature() {
  const uint64_t sz[] = {sizeof(DRule), sizeof(DVarRef), sizeof(DExc), sizeof(DOp), sizeof(DAction),
                         sizeof(DTmplPart), sizeof(DTmpl), sizeof(DDfa), sizeof(DStream), sizeof(DFilter),
                         sizeof(DJob), sizeof(DJobDfa), sizeof(DPat), sizeof(DScanVal), sizeof(Scalars),
                         sizeof(DNfa), sizeof(DPike), sizeof(DPikeInst), sizeof(DDynSite), sizeof(DSnapSlot)};
  return fnv64((const uint8_t*)sz, sizeof(sz));
}

struct Writer {
  std::vector<uint8_t> b;
  uint32_t n = 0;
  void raw(const void* p, size_t k) {
    const uint8_t* q = (const uint8_t*)p;
    b.insert(b.end(), q, q + k);
  }
  void section(uint32_t tag, uint32_t esz, uint64_t count, const void* p) {
    raw(&tag, 4);
    raw(&esz, 4);
    raw(&count, 8);
    if (count) raw(p, esz * count);
    while (b.size() % 8) b.push_back(0);
    n++;
  }
  template <class T>
  void vec(uint32_t tag, const std::vector<T>& v) {
    section(tag, (uint32_t)sizeof(T), v.size(), v.data());
  }
};

}  // namespace

std::vector<uint8_t> serialize_program(const Program& P) {
  Writer w;
#define X(tag, m) w.vec(tag, P.m);
  GI_ART_VECTORS(X)
#undef X
  Scalars s{};
  memcpy(s.item_sides, P.item_sides, 8);
  s.item_singles = P.item_singles;
  s.n_hit_slots = P.n_hit_slots;
  s.n_union_dfas = P.n_union_dfas;
  s.max_img_bytes = P.max_img_bytes;
  s.max_big_img_bytes = P.max_big_img_bytes;
  s.n_slots = P.n_slots;
  s.n_markers = P.n_markers;
  s.rule_engine = P.rule_engine;
  s.body_access = P.body_access;
  s.mv_used = P.mv_used;
  s.body_partial = P.body_partial;
  s.fold_on = P.fold_on;
  s.fold_nids = P.fold_nids;
  s.max_tx_lit = P.max_tx_lit;
  s.n_rm_groups = P.n_rm_groups;
  s.args_limit = P.args_limit;
  s.body_limit = P.body_limit;
  s.source_digest = P.source_digest;
  s.compiler_rev = compiler_rev_hash();
  w.section(kTagScalars, sizeof(Scalars), 1, &s);
  w.section(kTagPlan, 1, P.plan_json.size(), P.plan_json.data());
  std::string names;
  for (const auto& e : P.export_names) names.append(e).push_back('\0');
  w.section(kTagExportNames, 1, names.size(), names.data());

  std::vector<uint8_t> out(40);
  memcpy(out.data(), kMagic, 8);
  const uint32_t ver = kArtifactVersion, nsec = w.n;
  const uint64_t plen = w.b.size(), sum = fnv64(w.b.data(), w.b.size()), sig = layout_signature();
  memcpy(out.data() + 8, &ver, 4);
  memcpy(out.data() + 12, &nsec, 4);
  memcpy(out.data() + 16, &plen, 8);
  memcpy(out.data() + 24, &sum, 8);
  memcpy(out.data() + 32, &sig, 8);
  out.insert(out.end(), w.b.begin(), w.b.end());
  return out;
}

bool deserialize_program(const uint8_t* buf, size_t n, Program* P, std::string* err) {
  auto bad = [&](const std::string& m) {
    *err = "invalid GPU artifact: " + m;
    return false;
  };
  if (!buf || n < 40) return bad("truncated header");
  if (memcmp(buf, kMagic, 8) != 0) return bad("bad magic");
  uint32_t ver, nsec;
  uint64_t plen, sum, sig;
  memcpy(&ver, buf + 8, 4);
  memcpy(&nsec, buf + 12, 4);
  memcpy(&plen, buf + 16, 8);
  memcpy(&sum, buf + 24, 8);
  memcpy(&sig, buf + 32, 8);
  if (ver != kArtifactVersion) return bad("version " + std::to_string(ver) + " (this build reads " +
                                          std::to_string(kArtifactVersion) + ")");
  if (sig != layout_signature()) return bad("record layout of another build");
  if (plen != n - 40) return bad("payload length");
  if (fnv64(buf + 40, plen) != sum) return bad("checksum mismatch");
  Program out;
  bool seen_scalars = false;
  size_t off = 40;
  for (uint32_t k = 0; k < nsec; k++) {
    if (off + 16 > n) return bad("truncated section header");
    uint32_t tag, esz;
    uint64_t cnt;
    memcpy(&tag, buf + off, 4);
    memcpy(&esz, buf + off + 4, 4);
    memcpy(&cnt, buf + off + 8, 8);
    off += 16;
    if (esz == 0 || cnt > (n - off) / esz) return bad("section " + std::to_string(tag) + " out of range");
    const uint8_t* p = buf + off;
    const size_t bytes = (size_t)(esz * cnt);
    bool known = true;
    switch (tag) {
#define X(t, m)                                                                  \
  case t: {                                                                      \
    using T = typename decltype(out.m)::value_type;                              \
    if (esz != sizeof(T)) return bad("section " #m " record size");              \
    out.m.resize(cnt);                                                           \
    if (cnt) memcpy((void*)out.m.data(), p, bytes);                              \
    break;                                                                       \
  }
      GI_ART_VECTORS(X)
#undef X
      case kTagScalars: {
        if (esz != sizeof(Scalars) || cnt != 1) return bad("scalars");
        Scalars s;
        memcpy(&s, p, sizeof(s));
        if (s.compiler_rev != compiler_rev_hash()) return bad("written by another compiler revision");
        memcpy(out.item_sides, s.item_sides, 8);
        out.item_singles = s.item_singles;
        out.n_hit_slots = s.n_hit_slots;
        out.n_union_dfas = s.n_union_dfas;
        out.max_img_bytes = s.max_img_bytes;
        out.max_big_img_bytes = s.max_big_img_bytes;
        out.n_slots = s.n_slots;
        out.n_markers = s.n_markers;
        out.rule_engine = s.rule_engine;
        out.body_access = s.body_access;
        out.mv_used = s.mv_used;
        out.body_partial = s.body_partial;
        out.fold_on = s.fold_on;
        out.fold_nids = s.fold_nids;
        out.max_tx_lit = s.max_tx_lit;
        out.n_rm_groups = s.n_rm_groups;
        out.args_limit = s.args_limit;
        out.body_limit = s.body_limit;
        out.source_digest = s.source_digest;
        seen_scalars = true;
        break;
      }
      case kTagPlan:
        out.plan_json.assign((const char*)p, bytes);
        break;
      case kTagExportNames: {
        size_t a = 0;
        for (size_t i = 0; i < bytes; i++)
          if (p[i] == 0) {
            out.export_names.emplace_back((const char*)p + a, i - a);
            a = i + 1;
          }
        break;
      }
      default:
        known = false;
    }
    if (!known) return bad("unknown section " + std::to_string(tag));
    off += (bytes + 7) & ~(size_t)7;
    if (off > n) return bad("section padding");
  }
  if (!seen_scalars) return bad("no scalars section");
  if (off != n) return bad("trailing bytes");
  if (out.exports.size() != out.export_names.size()) return bad("exports");
  // cross-references the kernels trust: indices must stay inside their tables
  std::string verr;
  if (!validate_program(out, &verr)) return bad(verr);
  *P = std::move(out);
  return true;
}

bool validate_program(const Program& P, std::string* err) {
  auto bad = [&](const std::string& m) {
    *err = m;
    return false;
  };
  auto in = [](uint64_t off, uint64_t len, size_t size) { return off <= size && len <= size - off; };
  const size_t nrules = P.rules.size(), ndfa = P.dfas.size(), nstr = P.strpool.size(), ntm = P.tmpls.size();
  const uint32_t nslot = P.n_slots, nhit = P.n_hit_slots;
  if (P.slot_names.size() < 2ull * nslot) return bad("slot names");
  for (uint32_t s = 0; s < nslot; s++)
    if (!in(P.slot_names[2 * s], P.slot_names[2 * s + 1], nstr)) return bad("slot name range");
  if (P.exports.size() > GI_MAX_EXPORTS) return bad("export count");
  for (int32_t x : P.exports)
    if (x >= (int32_t)nslot) return bad("export slot");
  if (P.item_singles >> S_COUNT) return bad("item singles");
  // automata
  for (size_t i = 0; i < ndfa; i++) {
    const DDfa& d = P.dfas[i];
    if (d.n_states == 0 || d.n_states > 32768 || d.n_classes == 0 || d.n_classes > 256 || d.start >= d.n_states)
      return bad("automaton shape");
    const uint64_t nt = (uint64_t)d.n_states * d.n_classes;
    if (!in(d.trans_off, nt, P.trans.size())) return bad("automaton transitions");
    for (uint64_t k = 0; k < nt; k++) {
      const uint32_t nx = d.multi ? (P.trans[d.trans_off + k] & 0x7FFFu) : P.trans[d.trans_off + k];
      if (nx >= d.n_states) return bad("automaton transition target");
    }
    const uint32_t amn = d.byte_mode ? 256 : 128;
    if (!in(d.amap_off, amn, P.u8pool.size())) return bad("automaton class map");
    for (uint32_t k = 0; k < amn; k++)
      if (P.u8pool[d.amap_off + k] >= d.n_classes) return bad("automaton class");
    if (!in(d.nr_off, 3ull * d.nr_cnt, P.nranges.size())) return bad("automaton rune ranges");
    for (uint32_t k = 0; k < d.nr_cnt; k++)
      if (P.nranges[d.nr_off + 3 * k + 2] >= d.n_classes) return bad("automaton rune class");
    if (d.nonascii_cls >= d.n_classes) return bad("automaton non-ASCII class");
    if (d.multi) {
      if (!in(d.combo_off, d.n_classes, P.u8pool.size())) return bad("automaton combos");
      for (uint32_t k = 0; k < d.n_classes; k++)
        if (P.u8pool[d.combo_off + k] > 4) return bad("automaton combo");
      if (!in(d.acc_off, 5ull * d.n_states, P.u64pool.size())) return bad("automaton accept masks");
    } else if (!in(d.endacc_off, d.n_states, P.u8pool.size())) {
      return bad("automaton end accept");
    }
  }
  auto single_dfa = [&](int32_t id) { return id >= 0 && (size_t)id < ndfa && !P.dfas[id].multi; };
  for (const DNfa& f : P.nfas) {
    const uint64_t W = f.words;
    if (W == 0 || W > GI_NFA_MAX_WORDS || (uint64_t)f.n_pos + 1 > 64 * W || f.n_classes == 0 || f.n_classes > 256)
      return bad("nfa shape");
    if (!in(f.amap_off, 128, P.u8pool.size()) || !in(f.combo_off, f.n_classes, P.u8pool.size()) ||
        !in(f.nr_off, 3ull * f.nr_cnt, P.nranges.size()) || !in(f.cm_off, f.n_classes * W, P.u64pool.size()) ||
        !in(f.follow_off, ((uint64_t)f.n_pos + 1) * 16 * W, P.u64pool.size()))
      return bad("nfa tables");
    for (uint32_t k = 0; k < 128; k++)
      if (P.u8pool[f.amap_off + k] >= f.n_classes) return bad("nfa class");
    for (uint32_t k = 0; k < f.nr_cnt; k++)
      if (P.nranges[f.nr_off + 3 * k + 2] >= f.n_classes) return bad("nfa rune class");
  }
  // templates
  for (const DTmpl& t : P.tmpls)
    if (!in(t.part_begin, t.part_count, P.tparts.size())) return bad("template parts");
  for (const DTmplPart& p : P.tparts) {
    if (p.kind == TP_TX && (p.slot < 0 || (uint32_t)p.slot >= nslot)) return bad("template TX slot");
    if (p.kind == TP_SINGLE && p.single >= S_COUNT) return bad("template variable");
    if ((p.kind == TP_LIT || p.kind == TP_HEADER) && !in(p.off, p.len, nstr)) return bad("template string");
  }
  // rule records
  for (uint32_t t : P.top)
    if (t >= nrules) return bad("top-level rule index");
  for (const DRule& r : P.rules) {
    if (!in(r.var_begin, r.var_count, P.vars.size()) || (r.op >= 0 && (uint32_t)r.op >= P.ops.size()) ||
        !in(r.act_begin, r.act_count, P.acts.size()) || !in(r.tchain_off, r.tchain_len, P.tchains.size()) ||
        (r.chain_next >= 0 && (uint32_t)r.chain_next >= nrules) || r.phase > 5 ||
        (r.hit_slot >= 0 && (uint32_t)r.hit_slot >= nhit) || r.hit_slot < -1 || r.disruptive > D_ALLOW_REQUEST)
      return bad("rule record out of range");
    // k_eval runs the link's capture program (run_capture reads P.pikes[op.pike] and the
    // request's capture workspace): only an @rx link with a program may carry the flag
    if ((r.flags & RF_CAPTURE) &&
        (r.op < 0 || P.ops[r.op].kind != OP_RX || P.ops[r.op].pike < 0))
      return bad("capture flag without a capture program");
  }
  // folded prefix (compile.cpp fold_program): snapshot per slot, ids, resume point
  if (P.tx_snap.size() != nslot) return bad("TX snapshot size");
  for (const DSnapSlot& z : P.tx_snap)
    if (z.state > 2 || (z.state == 2 && !in(z.off, z.len, nstr))) return bad("TX snapshot value");
  if (P.fold_nids > P.fold_ids.size()) return bad("folded ids");
  if (P.fold_runs.size() % 4) return bad("folded runs");
  for (size_t q = 0; q + 3 < P.fold_runs.size(); q += 4)
    if ((uint64_t)P.fold_runs[q] + P.fold_runs[q + 1] > P.fold_nids ||
        (P.fold_runs[q + 3] != 0xFFFFFFFFu && P.fold_runs[q + 3] >= P.n_markers))
      return bad("folded run");
  for (const DRule& r : P.rules)
    if ((r.flags & RF_FOLDED) && (4ull * r._pad2 + 3 >= P.fold_runs.size() || (r.flags & RF_CHILD)))
      return bad("folded rule");
  for (const DRule& r : P.rules)
    if ((r.flags & RF_CONST) && r.op >= 0 && r.var_count == 0) return bad("constant link without targets");
  for (uint32_t t : P.body_links)
    if (t >= nrules || P.rules[t].op < 0 || P.rules[t].hit_slot < 0) return bad("body link");
  for (const DVarRef& v : P.vars) {
    if (v.key_mode == 1 && !in(v.key_off, v.key_len, nstr)) return bad("variable key");
    if (v.key_mode == 2 && !single_dfa(v.key_dfa)) return bad("variable key automaton");
    if (v.key_mode > 2) return bad("variable key mode");
    if (!in(v.exc_begin, v.exc_count, P.excs.size())) return bad("variable exceptions");
    if (v.var == V_TX && v.key_mode != 2 && v.slot >= (int32_t)nslot) return bad("variable TX slot");
    if (v.pre_len && (v.var != V_TX || v.key_mode != 2 || v.slot < 0 || !in((uint32_t)v.slot, v.pre_len, nstr)))
      return bad("TX key prefix");
    if (v.var == V_TX && v.key_mode == 2) {  // static slots the key regex matches
      if (!in(v.key_off, v.key_len, P.txrx.size())) return bad("TX regex slot list");
      for (uint32_t k = 0; k < v.key_len; k++)
        if (P.txrx[v.key_off + k] >= nslot) return bad("TX regex slot");
    }
  }
  for (const DExc& x : P.excs) {
    if (x.dfa >= 0 ? !single_dfa(x.dfa) : !in(x.off, x.len, nstr)) return bad("exception");
  }
  for (const DOp& o : P.ops) {
    if ((o.kind == OP_RX || o.kind == OP_PM) && !single_dfa(o.dfa) && o.nfa < 0) return bad("operator automaton");
    if (o.dfa >= 0 && !single_dfa(o.dfa)) return bad("operator automaton index");
    if (o.ngroups && (o.dfa < 0 || (uint64_t)o.dfa + o.ngroups > P.dfas.size())) return bad("phrase groups");
    for (uint32_t g = 1; g < o.ngroups; g++)
      if (!single_dfa(o.dfa + (int32_t)g)) return bad("phrase group automaton");
    if (o.nfa >= 0 && (size_t)o.nfa >= P.nfas.size()) return bad("operator nfa index");
    if (o.tmpl >= 0 && (size_t)o.tmpl >= ntm) return bad("operator template");
    if (o.arg_is_lit && !in(o.lit_off, o.lit_len, nstr)) return bad("operator literal");
    if (o.pike >= 0 && ((size_t)o.pike >= P.pikes.size() || o.kind != OP_RX)) return bad("operator capture program");
    // the @ipMatch kernel path reads lit_len bytes of network records at lit_off
    if (o.kind == OP_IPMATCH && (!o.arg_is_lit || !in(o.lit_off, o.lit_len, nstr) || o.lit_len % GI_IPNET_BYTES))
      return bad("ipMatch networks");
  }
  for (const DAction& a : P.acts) {
    if (a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) {
      if (a.slot < -1 || (a.slot >= 0 && (uint32_t)a.slot >= nslot)) return bad("setvar slot");
      if (a.slot == -1 && (a.aux < 0 || (size_t)a.aux >= ntm || P.dyn_sites.empty())) return bad("setvar key template");
      if (a.tmpl >= 0 && (size_t)a.tmpl >= ntm) return bad("setvar template");
      if ((a.a == SV_ADD_SLOT || a.a == SV_SUB_SLOT) && (a.b < 0 || (uint64_t)a.b >= nslot)) return bad("setvar source");
    }
    if (a.kind == A_CTL_RULE_REMOVE_TARGET && (a.tmpl < 0 || a.aux < 0 || !in((uint32_t)a.tmpl, (uint32_t)a.aux, nstr)))
      return bad("ctl target key");
    if ((a.kind == A_CTL_RULE_REMOVE_GROUP && (a.a < 0 || a.a >= (int64_t)P.n_rm_groups)) ||
        (a.kind == A_CTL_RULE_REMOVE_TARGET && a.a == GI_RM_GROUP_MODE && (a.b < 0 || a.b >= (int64_t)P.n_rm_groups)))
      return bad("ctl removal group");
  }
  if (P.n_rm_groups > GI_MAX_RM_GROUPS || P.rule_groups.size() != std::max<size_t>(nrules, 1)) return bad("removal groups");
  for (uint32_t m : P.rule_groups)
    if (P.n_rm_groups < 32 && (m >> P.n_rm_groups)) return bad("rule removal group mask");
  {
  }
  // capture programs (pike.h): every jump inside its program, rune ranges in the pool
  for (const DPike& k : P.pikes) {
    if (!in(k.inst_off, k.n_inst, P.pike_insts.size()) || k.n_inst == 0 || k.start >= k.n_inst ||
        k.nslot < 2 || k.nslot > GI_PIKE_MAX_SLOTS || (k.nslot & 1) || k.whole > 1 || (k.whole && k.nslot != 2))
      return bad("capture program");
    for (uint32_t i = 0; i < k.n_inst; i++) {
      const DPikeInst& I = P.pike_insts[k.inst_off + i];
      if (I.op < PK_RUNE || I.op > PK_FAIL) return bad("capture instruction");
      if ((I.op != PK_MATCH && I.op != PK_FAIL && I.x >= k.n_inst) || (I.op == PK_SPLIT && I.y >= k.n_inst))
        return bad("capture jump");
      if (I.op == PK_RUNE && !in(I.roff, 2ull * I.rcnt, P.pike_ranges.size())) return bad("capture rune ranges");
    }
  }
  // phase-A scan plan
  if (P.streams.size() > GI_MAX_STREAMS || P.filters.size() > GI_MAX_GFILTERS) return bad("scan plan size");
  const uint32_t ngf = (uint32_t)P.filters.size();
  for (const DFilter& f : P.filters) {
    if (f.single != GI_NO_SINGLE && f.single >= S_COUNT) return bad("filter variable");
    if (f.key_mode == 1 && !in(f.key_off, f.key_len, nstr)) return bad("filter key");
    if (f.key_mode == 2 && !single_dfa(f.key_dfa)) return bad("filter key automaton");
    if (!in(f.exc_begin, f.exc_count, P.excs.size())) return bad("filter exceptions");
  }
  for (uint8_t g : P.sfilt)
    if (g >= ngf) return bad("stream filter id");
  for (const DStream& s : P.streams) {
    if (!in(s.tchain_off, s.tchain_len, P.tchains.size()) || !in(s.filt_begin, s.filt_count, P.sfilt.size()) ||
        !in(s.job_begin, s.job_count, P.jobs.size()) || !in(s.val_begin, s.val_count, P.svals.size()))
      return bad("stream record");
    if (s.det_id != 0xFF && s.det_id >= GI_MAX_DET_STREAMS) return bad("stream detect id");  // k_stream shifts by it
    if (!in(s.rmap_off, 3ull * s.rmap_cnt, P.nranges.size())) return bad("stream rune map");
    for (uint32_t k = 0; k < s.rmap_cnt; k++)
      if (P.nranges[s.rmap_off + 3 * k + 2] < 0x80 || P.nranges[s.rmap_off + 3 * k + 2] > 0xFF) return bad("stream rune map byte");
  }
  for (const DScanVal& v : P.svals)
    if (v.slot >= nhit) return bad("validate slot");
  for (const DPat& p : P.pats)
    if (p.slot >= nhit) return bad("pattern slot");
  for (uint32_t s : P.always_slots)
    if (s >= nhit) return bad("always slot");
  if (P.max_img_bytes > GI_JOB_LDS_BYTES || P.max_big_img_bytes > GI_BIG_LDS_BYTES + 4096) return bad("image limits");
  for (const DJob& J : P.jobs) {
    if (J.stream >= P.streams.size() || !in(J.img_off, J.img_bytes, P.images.size()) ||
        !in(J.jdfa_begin, J.jdfa_count, P.jdfas.size()) || J.jdfa_count == 0 || J.jdfa_count > GI_JOB_MAX_DFA)
      return bad("job record");
    if (J.lds && J.img_bytes > (J.big ? P.max_big_img_bytes : P.max_img_bytes)) return bad("job image size");
    const uint8_t* img = P.images.data() + J.img_off;
    if (!in(J.lds_fmask, 8ull * J.jdfa_count * ngf, J.img_bytes) || J.img_bytes < 4 * 129) return bad("job fmask table");
    for (uint32_t q = 0; q < J.jdfa_count; q++) {
      const DJobDfa& jd = P.jdfas[J.jdfa_begin + q];
      if (jd.dfa < 0 || (size_t)jd.dfa >= ndfa) return bad("job automaton");
      const DDfa& d = P.dfas[jd.dfa];
      if (jd.n_pat == 0 || jd.n_pat > 64 || !in(jd.pat_begin, jd.n_pat, P.pats.size()) ||
          !in(jd.fmask_off, ngf, P.u64pool.size()))
        return bad("job automaton patterns");
      const uint64_t pm = jd.n_pat == 64 ? ~0ull : (1ull << jd.n_pat) - 1;
      if (jd.neg_mask & ~pm) return bad("job negation mask");
      for (uint32_t g = 0; g < ngf; g++) {
        uint64_t m;
        memcpy(&m, img + J.lds_fmask + 8ull * (q * ngf + g), 8);
        if ((m | P.u64pool[jd.fmask_off + g]) & ~pm) return bad("job filter mask");
      }
      if (!J.lds) continue;
      const uint64_t tb = 2ull * d.n_states * d.n_classes;
      if (jd.lds_trans < 0 || !in((uint32_t)jd.lds_trans, tb, J.img_bytes) || (jd.lds_trans & 1)) return bad("image transitions");
      if (jd.lds_endacc < 0 || !in((uint32_t)jd.lds_endacc, (d.multi ? 8ull : 1ull) * d.n_states, J.img_bytes) ||
          (d.multi && (jd.lds_endacc & 7)))
        return bad("image end accept");
      if (jd.lds_slots < 0 || !in((uint32_t)jd.lds_slots, 4ull * jd.n_pat, J.img_bytes) || (jd.lds_slots & 3))
        return bad("image slots");
      if (d.multi && (jd.lds_combo < 0 || !in((uint32_t)jd.lds_combo, d.n_classes, J.img_bytes))) return bad("image combos");
      for (uint64_t k = 0; k < (uint64_t)d.n_states * d.n_classes; k++) {
        uint16_t tv;
        memcpy(&tv, img + jd.lds_trans + 2 * k, 2);
        if ((d.multi ? (tv & 0x7FFFu) : tv) >= d.n_states) return bad("image transition target");
      }
      for (uint32_t c = 0; c <= 128; c++) {
        uint32_t jm;
        memcpy(&jm, img + 4 * c, 4);
        if (((jm >> (8 * q)) & 0xFFu) >= d.n_classes) return bad("image joint class map");
      }
      if (d.multi)
        for (uint32_t c = 0; c < d.n_classes; c++)
          if (img[jd.lds_combo + c] > 4) return bad("image combo");
      for (uint32_t k = 0; k < jd.n_pat; k++) {
        uint32_t sl;
        memcpy(&sl, img + jd.lds_slots + 4 * k, 4);
        if (sl >= nhit) return bad("image slot");
      }
    }
  }
  return true;
}

}  // namespace gi
