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
  uint8_t rule_engine, body_access, _pad[6];
  uint64_t body_limit, source_digest;
};

// One entry per Program vector: tag, member.  Order = file order.
#define GI_ART_VECTORS(X)                                                                                     \
  X(1, rules) X(2, top) X(3, vars) X(4, excs) X(5, ops) X(6, acts) X(7, tparts) X(8, tmpls) X(9, tchains)    \
  X(10, dfas) X(11, trans) X(12, u8pool) X(13, nranges) X(14, strpool) X(15, slot_names) X(16, u64pool)     \
  X(17, streams) X(18, filters) X(19, sfilt) X(20, body_links) X(21, always_slots) X(22, jobs) X(23, jdfas) \
  X(24, pats) X(25, svals) X(26, images) X(27, exports)

constexpr uint32_t kTagScalars = 100, kTagPlan = 101, kTagExportNames = 102;

uint64_t layout_signature() {
  const uint64_t sz[] = {sizeof(DRule), sizeof(DVarRef), sizeof(DExc), sizeof(DOp), sizeof(DAction),
                         sizeof(DTmplPart), sizeof(DTmpl), sizeof(DDfa), sizeof(DStream), sizeof(DFilter),
                         sizeof(DJob), sizeof(DJobDfa), sizeof(DPat), sizeof(DScanVal), sizeof(Scalars)};
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
  s.body_limit = P.body_limit;
  s.source_digest = P.source_digest;
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
  // cross-references the kernels trust: indices must stay inside their tables
  for (uint32_t t : out.top)
    if (t >= out.rules.size()) return bad("top-level rule index");
  for (uint32_t t : out.body_links)
    if (t >= out.rules.size()) return bad("body link index");
  for (const DRule& r : out.rules) {
    if ((uint64_t)r.var_begin + r.var_count > out.vars.size() || (r.op >= 0 && (uint32_t)r.op >= out.ops.size()) ||
        (uint64_t)r.act_begin + r.act_count > out.acts.size() ||
        (uint64_t)r.tchain_off + r.tchain_len > out.tchains.size() ||
        (r.chain_next >= 0 && (uint32_t)r.chain_next >= out.rules.size()))
      return bad("rule record out of range");
  }
  if (out.exports.size() != out.export_names.size()) return bad("exports");
  *P = std::move(out);
  return true;
}

}  // namespace gi
