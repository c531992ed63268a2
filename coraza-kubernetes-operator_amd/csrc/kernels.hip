// HIP kernels of the inspection engine (gfx950).
//
// v1 pipeline = one launch, one thread per request ("transaction lane"):
//   collect  : ProcessURI + AddRequestHeader (query/cookie parsing, Go
//              net/url re-encoding of REQUEST_URI) into a per-request field
//              table in HBM scratch
//   phase 1  : RuleGroup.Eval(1) -- the rule interpreter below
//   body     : ProcessRequestBody (URLENCODED / JSON -> ARGS_POST)
//   phase 2  : RuleGroup.Eval(2)
//   verdict  : Interruption + matched rule ids + exported TX scores,
//              block-reduced tallies (one atomic per block per counter)
// Semantics follow coraza/v3 v3.3.3 [upstream, see DESIGN.md]; every
// function names the coraza source it restates.
// (built with -D__HIP_DEFINE_EXTENDED_HOST_MIN_MAX__=1: the host interpreter,
// cpu_inspect_one, needs min/max over every integer type, as on the device)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "gi_kernels.h"
#include "html_entities.h"
#include "libinj.h"

// k_detect's own copy of the detectors (libinj_body.h again, in gi::lid): its
// out-of-line functions are called by k_detect alone, so they are compiled
// for k_detect's register budget instead of the largest one among k_eval /
// k_stream / k_long, which share the gi:: copy.
namespace gi {
namespace lid {
// the keyword tables in k_detect's LDS (loaded at its start): every word
// lookup is a hash probe + compare there, and the lane state needs no pointers
__shared__ uint32_t li_lw[LI_NWORDS];
__shared__ uint16_t li_lh[LI_HASH_SIZE];
__shared__ __attribute__((aligned(16))) uint8_t li_lp[sizeof(kLiPool)];
#define LI_LDS_TABLES (LiTables{li_lw, li_lp, li_lh})
#include "libinj_body.h"
#undef LI_LDS_TABLES
}  // namespace lid
}  // namespace gi

namespace gi {

// ------------------------------------------------------------ small utils
struct Str {
  const uint8_t* p;
  uint32_t n;
};

struct Field {
  const uint8_t* k;
  const uint8_t* v;
  uint32_t kn, vn;
  uint32_t kind;
  uint32_t _pad;
};

struct Slot {  // 16 B: a wave's slot-s accesses cover 1 KB (k_eval's TX traffic)
  union {
    int64_t num;       // state 1
    const uint8_t* p;  // state 2 (n bytes)
  };
  uint32_t n;
  uint32_t state;  // 0 unset, 1 integer (canonical decimal), 2 string
};
static_assert(sizeof(Slot) == GI_SLOT_BYTES, "Slot size (runtime.cpp sizes txslots with it)");

GI_TABLE uint8_t kConstStrs[] =
    "0\0URLENCODED\0JSON\0XML\0MULTIPART\0" "1\0JSON: invalid JSON\0" "//@*\0/*\0\0\0\0\0\0\0\0";  // padded for load_u32u
#define CS_ZERO (kConstStrs + 0)
#define CS_URLENCODED (kConstStrs + 2)
#define CS_JSON (kConstStrs + 13)
#define CS_XML (kConstStrs + 18)
#define CS_MULTIPART (kConstStrs + 22)
#define CS_ONE (kConstStrs + 32)
#define CS_JSON_ERR (kConstStrs + 34)
#define CS_XML_ATTRS (kConstStrs + 53)  // XML collection keys (xml.go: "//@*" attribute values, "/*" text)
#define CS_XML_TEXT (kConstStrs + 58)

GI_HD inline bool ishex(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
GI_HD inline uint8_t hexv(uint8_t c) {
  return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
}
GI_HD inline uint8_t x2c(uint8_t a, uint8_t b) { return (uint8_t)((hexv(a) << 4) | hexv(b)); }
GI_HD inline uint8_t alower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
GI_HD inline bool isalnum_(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}
GI_HD inline bool isws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

// Four bytes at p (any alignment) from two aligned dword loads: long values
// are read a word per load instead of a byte per load.  May read up to 7
// bytes past p (every buffer is padded: runtime.cpp).
GI_HD __forceinline__ uint32_t load_u32u(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  return sh ? __builtin_amdgcn_alignbyte(w[1], lo, sh) : lo;
#else
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
#endif
}

// LDS byte pointers (k_body's tiles): the transformations below are templates
// over their source / destination pointer types, so a tile's accesses are
// ds_* ops whether or not the compiler inlines them -- never FLAT ops on an
// LDS address (which the compiler may merge into misaligned wide stores).
typedef __attribute__((address_space(3))) uint8_t gi_lds_u8;
typedef __attribute__((address_space(3))) uint32_t gi_lds_u32;
__device__ __forceinline__ uint32_t load_u32u(const gi_lds_u8* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  const gi_lds_u32* w = (const gi_lds_u32*)(uintptr_t)(a & ~3u);
  const uint32_t sh = a & 3u;
  const uint32_t lo = w[0];
#if defined(__HIP_DEVICE_COMPILE__)
  return sh ? __builtin_amdgcn_alignbyte(w[1], lo, sh) : lo;
#else
  return sh ? (uint32_t)((((uint64_t)w[1] << 32) | lo) >> (8 * sh)) : lo;
#endif
}
__device__ __forceinline__ void store_u32a(gi_lds_u8* p, uint32_t v) { *(gi_lds_u32*)p = v; }
// a dword store at a 4-byte aligned address
GI_HD __forceinline__ void store_u32a(uint8_t* p, uint32_t v) { *(uint32_t*)p = v; }

// Word-at-a-time byte helpers for the interpreter's per-request strings
// (k_eval: one lane per request, so every byte access is a scattered memory
// instruction of its own).  Sources must be padded buffers (the batch data,
// the request scratch, the program's string pool: runtime.cpp pads each by
// >= 16 bytes) -- they may read up to 8 bytes past the end; never a stack array.
GI_HD __forceinline__ uint32_t tail_mask(uint32_t r) { return r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u; }
// ASCII 'A'-'Z' | 0x20 in each byte of x (other bytes unchanged)
GI_HD __forceinline__ uint32_t lower4(uint32_t x) {
  const uint32_t ge_a = (x & 0x7F7F7F7Fu) + 0x3F3F3F3Fu;  // bit 7: byte & 0x7F >= 'A'
  const uint32_t gt_z = (x & 0x7F7F7F7Fu) + 0x25252525u;  // bit 7: byte & 0x7F > 'Z'
  return x | (((ge_a ^ gt_z) & ~x & 0x80808080u) >> 2);
}
// n bytes s -> d (any alignments): the head up to d's dword alignment and the
// tail byte-wise, the rest one aligned dword store per 4 bytes.  A source on
// the stack (a number formatted into a local buffer) is copied byte-wise.
GI_HD __forceinline__ void copy_bytes(uint8_t* d, const uint8_t* s, uint32_t n) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (n) memcpy(d, s, n);
#else
  uint32_t i = 0;
  if (n >= 8 && !__builtin_amdgcn_is_private(s)) {
    const uint32_t head = (4u - ((uint32_t)(uintptr_t)d & 3u)) & 3u;
    for (; i < head; i++) d[i] = s[i];
    for (; i + 4 <= n; i += 4) *(uint32_t*)(d + i) = load_u32u(s + i);
  }
  for (; i < n; i++) d[i] = s[i];
#endif
}
// the same, ASCII-lowercasing
GI_HD __forceinline__ void copy_lower(uint8_t* d, const uint8_t* s, uint32_t n) {
  uint32_t i = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  if (n >= 8 && !__builtin_amdgcn_is_private(s)) {
    const uint32_t head = (4u - ((uint32_t)(uintptr_t)d & 3u)) & 3u;
    for (; i < head; i++) d[i] = alower(s[i]);
    for (; i + 4 <= n; i += 4) *(uint32_t*)(d + i) = lower4(load_u32u(s + i));
  }
#endif
  for (; i < n; i++) d[i] = alower(s[i]);
}
// byte equality of two padded strings, a word per step
GI_HD __forceinline__ bool eq_bytes_w(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  if (an != bn) return false;
#if defined(__HIP_DEVICE_COMPILE__)
  for (uint32_t i = 0; i < an; i += 4)
    if ((load_u32u(a + i) ^ load_u32u(b + i)) & tail_mask(an - i)) return false;
  return true;
#else
  return an == 0 || memcmp(a, b, an) == 0;
#endif
}
// gi_fnv1a(s, n, false) over a padded string, a word loaded per 4 bytes
GI_HD __forceinline__ uint32_t fnv1a_w(const uint8_t* s, uint32_t n) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return gi_fnv1a(s, n, false);
#endif
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; i += 4) {
    const uint32_t x = load_u32u(s + i);
    const uint32_t m = n - i < 4 ? n - i : 4u;
    for (uint32_t k = 0; k < m; k++) h = (h ^ ((x >> (8 * k)) & 0xFFu)) * 16777619u;
  }
  return h;
}

GI_HD __forceinline__ bool eq_bytes(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  if (an != bn) return false;
  for (uint32_t i = 0; i < an; i++)
    if (a[i] != b[i]) return false;
  return true;
}
GI_HD bool eq_ascii_ci_both(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (alower(a[i]) != alower(b[i])) return false;
  return true;
}
GI_HD __forceinline__ bool eq_ascii_ci(const uint8_t* a, uint32_t an, const uint8_t* lowered, uint32_t bn) {
  if (an != bn) return false;
  for (uint32_t i = 0; i < an; i++)
    if (alower(a[i]) != lowered[i]) return false;
  return true;
}
GI_HD int64_t find_bytes(const uint8_t* h, uint32_t hn, const uint8_t* nd, uint32_t nn) {
  if (nn == 0) return 0;
  if (nn > hn) return -1;
  for (uint32_t i = 0; i + nn <= hn; i++) {
    uint32_t k = 0;
    while (k < nn && h[i + k] == nd[k]) k++;
    if (k == nn) return i;
  }
  return -1;
}

// strconv.Atoi: ok=false on syntax error; saturates on range error.
GI_HD int64_t go_atoi(const uint8_t* s, uint32_t n, bool* ok) {
  uint32_t i = 0;
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) {
    neg = s[i] == '-';
    i++;
  }
  if (i >= n) {
    *ok = false;
    return 0;
  }
  uint64_t acc = 0;
  bool ovf = false;
  for (; i < n; i++) {
    uint8_t c = s[i];
    if (c < '0' || c > '9') {
      *ok = false;
      return 0;
    }
    if (acc > (UINT64_MAX - 9) / 10) ovf = true;
    else acc = acc * 10 + (c - '0');
  }
  if (!neg && (ovf || acc > (uint64_t)INT64_MAX)) {
    *ok = false;
    return INT64_MAX;
  }
  if (neg && (ovf || acc > (uint64_t)INT64_MAX + 1)) {
    *ok = false;
    return INT64_MIN;
  }
  *ok = true;
  return neg ? (int64_t)(0 - acc) : (int64_t)acc;
}

// strconv.Itoa into buf (>= 21 bytes), returns length.
GI_HD __forceinline__ uint32_t go_itoa(int64_t v, uint8_t* buf) {
  uint8_t tmp[24];
  uint32_t n = 0;
  uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  do {
    tmp[n++] = (uint8_t)('0' + u % 10);
    u /= 10;
  } while (u);
  uint32_t k = 0;
  if (v < 0) buf[k++] = '-';
  while (n) buf[k++] = tmp[--n];
  return k;
}

// utf8.DecodeRune
template <class S>
GI_HD __forceinline__ uint32_t decode_rune(S b, uint32_t n, uint32_t i, uint32_t* w) {
  uint8_t c0 = b[i];
  if (c0 < 0x80) {
    *w = 1;
    return c0;
  }
  uint32_t need;
  uint8_t lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) need = 1;
  else if (c0 == 0xE0) { need = 2; lo = 0xA0; }
  else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) need = 2;
  else if (c0 == 0xED) { need = 2; hi = 0x9F; }
  else if (c0 == 0xF0) { need = 3; lo = 0x90; }
  else if (c0 >= 0xF1 && c0 <= 0xF3) need = 3;
  else if (c0 == 0xF4) { need = 3; hi = 0x8F; }
  else { *w = 1; return 0xFFFD; }
  if (n - i < need + 1) { *w = 1; return 0xFFFD; }
  uint8_t c1 = b[i + 1];
  if (c1 < lo || c1 > hi) { *w = 1; return 0xFFFD; }
  for (uint32_t k = 2; k <= need; k++) {
    uint8_t ck = b[i + k];
    if (ck < 0x80 || ck > 0xBF) { *w = 1; return 0xFFFD; }
  }
  *w = need + 1;
  if (need == 1) return ((c0 & 0x1F) << 6) | (c1 & 0x3F);
  if (need == 2) return ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (b[i + 2] & 0x3F);
  return ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6) | (b[i + 3] & 0x3F);
}

template <class D>
GI_HD __forceinline__ uint32_t encode_rune(uint32_t r, D o) {
  if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
  if (r < 0x800) { o[0] = 0xC0 | (r >> 6); o[1] = 0x80 | (r & 0x3F); return 2; }
  if (r < 0x10000) {
    o[0] = 0xE0 | (r >> 12); o[1] = 0x80 | ((r >> 6) & 0x3F); o[2] = 0x80 | (r & 0x3F);
    return 3;
  }
  o[0] = 0xF0 | (r >> 18); o[1] = 0x80 | ((r >> 12) & 0x3F); o[2] = 0x80 | ((r >> 6) & 0x3F);
  o[3] = 0x80 | (r & 0x3F);
  return 4;
}

// bit scans the interpreter uses on both targets
GI_HD __forceinline__ int gi_ffsll(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll((unsigned long long)x);
#else
  return __builtin_ffsll((long long)x);
#endif
}
// profiling counters / lane identity (GI_PROF diagnostics): nothing on the host interpreter
GI_HD __forceinline__ uint64_t gi_clock() {
#if defined(__HIP_DEVICE_COMPILE__)
  return clock64();
#else
  return 0;
#endif
}
// a list slot (the gate's pending list; the host interpreter never appends)
GI_HD __forceinline__ uint32_t gi_fetch_add(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  const uint32_t o = *p;
  *p = o + v;
  return o;
#endif
}
GI_HD __forceinline__ void gi_prof_add(unsigned long long* p, unsigned long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
GI_HD __forceinline__ uint32_t gi_tid() {
#if defined(__HIP_DEVICE_COMPILE__)
  return threadIdx.x;
#else
  return 0;
#endif
}
GI_HD __forceinline__ int gi_popcll(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll((unsigned long long)x);
#else
  return __builtin_popcountll((unsigned long long)x);
#endif
}

// --------------------------------------------------------------- DFA scan
// Sticky-accept DFA over rune classes (rune mode: Go UTF-8 decoding) or
// bytes (phrase automata).  fold: ASCII-lowercase bytes before the lookup.
GI_HD bool dfa_match(const DProgram& P, int32_t id, const uint8_t* s, uint32_t n, bool fold) {
  const DDfa d = P.dfas[id];
  const uint16_t* __restrict__ tr = P.trans + d.trans_off;
  const uint8_t* __restrict__ amap = P.u8pool + d.amap_off;
  const uint32_t ncls = d.n_classes;
  uint32_t st = d.start;
  uint32_t i = 0;
  uint32_t win = 0, wbeg = 0, wend = 0;  // s[wbeg, wend) in win
  if (d.byte_mode) {
    while (i < n) {
      if (st == d.accept) return true;
      if (i >= wend) {
        win = load_u32u(s + i);
        wbeg = i;
        wend = i + 4;
      }
      uint8_t c = (uint8_t)(win >> (8 * (i - wbeg)));
      i++;
      if (fold) c = alower(c);
      st = tr[st * ncls + amap[c]];
    }
  } else {
    while (i < n) {
      if (st == d.accept) return true;
      if (i >= wend) {
        win = load_u32u(s + i);
        wbeg = i;
        wend = i + 4;
      }
      uint8_t c = (uint8_t)(win >> (8 * (i - wbeg)));
      uint32_t cls;
      if (c < 0x80) {
        if (fold) c = alower(c);
        cls = amap[c];
        i++;
      } else {
        uint32_t w;
        uint32_t r = decode_rune(s, n, i, &w);
        i += w;
        if (d.nonascii_uniform) {
          cls = d.nonascii_cls;
        } else {
          const uint32_t* nr = P.nranges + d.nr_off;
          uint32_t lo = 0, hi = d.nr_cnt;
          cls = 0;
          while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (nr[mid * 3 + 1] < r) lo = mid + 1;
            else hi = mid;
          }
          if (lo < d.nr_cnt && nr[lo * 3] <= r) cls = nr[lo * 3 + 2];
        }
      }
      st = tr[st * ncls + cls];
    }
  }
  return P.u8pool[d.endacc_off + st] != 0;
}

// Exact NFA simulation for an @rx whose DFA exceeds the state cap (regex.h
// NfaTables): T = positions consumed by the previous rune; before each rune
// the epsilon closure from T and from the start (unanchored search) is the
// union of precomputed rows for (previous, next) rune kinds, which is what
// ^ $ \b \B look at; a closure holding the match bit is a match.
GI_HD __noinline__ bool nfa_match(const DProgram& P, int32_t id, const uint8_t* s, uint32_t n) {
  const DNfa N = P.nfas[id];
  const uint32_t W = N.words;
  const uint8_t* amap = P.u8pool + N.amap_off;
  const uint8_t* combo = P.u8pool + N.combo_off;
  const uint32_t* nr = P.nranges + N.nr_off;
  const uint64_t* cm = P.u64pool + N.cm_off;
  const uint64_t* F = P.u64pool + N.follow_off;
  uint64_t T[GI_NFA_MAX_WORDS], S[GI_NFA_MAX_WORDS];
  for (uint32_t k = 0; k < W; k++) T[k] = 0;
  uint32_t prev = 0, i = 0;
  for (;;) {
    uint32_t cls = 0, next = 0, w = 1;
    if (i < n) {
      const uint8_t c = s[i];
      if (c < 0x80) {
        cls = amap[c];
      } else {
        const uint32_t r = decode_rune(s, n, i, &w);
        uint32_t lo = 0, hi = N.nr_cnt;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (nr[mid * 3 + 1] < r) lo = mid + 1;
          else hi = mid;
        }
        cls = (lo < N.nr_cnt && nr[lo * 3] <= r) ? nr[lo * 3 + 2] : 0u;
      }
      const uint8_t cb = combo[cls];
      next = (cb & 1) ? 1u : (cb & 2) ? 2u : 3u;
    }
    const uint32_t cmb = prev * 4 + next;
    const uint64_t* st = F + ((uint64_t)N.n_pos * 16 + cmb) * W;
    for (uint32_t k = 0; k < W; k++) S[k] = st[k];
    for (uint32_t k = 0; k < W; k++)
      for (uint64_t b = T[k]; b; b &= b - 1) {
        const uint64_t* row = F + ((uint64_t)(k * 64 + gi_ffsll(b) - 1) * 16 + cmb) * W;
        for (uint32_t j = 0; j < W; j++) S[j] |= row[j];
      }
    if ((S[N.n_pos >> 6] >> (N.n_pos & 63)) & 1) return true;
    if (i >= n) return false;
    const uint64_t* cr = cm + (uint64_t)cls * W;
    for (uint32_t k = 0; k < W; k++) T[k] = S[k] & cr[k];
    prev = next;
    i += w;
  }
}

// ----------------------------------------------------------- transforms
// Each writes dst (capacity cap) and returns the new length, or -1 on
// overflow.  [upstream coraza internal/transformations/*.go]

GI_HD uint32_t lower_rune(const DProgram& P, uint32_t r) {
  if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
  uint32_t lo = 0, hi = P.n_lower_pairs;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (P.lower_pairs[mid * 2] < r) lo = mid + 1;
    else hi = mid;
  }
  if (lo < P.n_lower_pairs && P.lower_pairs[lo * 2] == r) return P.lower_pairs[lo * 2 + 1];
  return r;
}

// Go strings.ToLower
template <class S, class D>
GI_HD int64_t t_lowercase(const DProgram& P, S s, uint32_t n, D d, uint32_t cap) {
  bool ascii = true;
  for (uint32_t i = 0; i < n && ascii; i += 4) {
    uint32_t x = load_u32u(s + i);
    if (n - i < 4) x &= (1u << (8 * (n - i))) - 1u;
    ascii = !(x & 0x80808080u);
  }
  if (ascii) {
    if (n > cap) return -1;
    if (!((uintptr_t)d & 3) && ((n + 3) & ~3u) <= cap) {  // SWAR: ASCII 'A'-'Z' | 0x20, a word at a time
      for (uint32_t i = 0; i < n; i += 4) {
        const uint32_t x = load_u32u(s + i);
        const uint32_t ge_a = (x & 0x7F7F7F7Fu) + 0x3F3F3F3Fu;  // bit 7: byte >= 'A'
        const uint32_t gt_z = (x & 0x7F7F7F7Fu) + 0x25252525u;  // bit 7: byte > 'Z'
        store_u32a(d + i, x | (((ge_a ^ gt_z) & ~x & 0x80808080u) >> 2));
      }
    } else {
      for (uint32_t i = 0; i < n; i++) d[i] = alower(s[i]);
    }
    return n;
  }
  uint32_t o = 0, i = 0;
  while (i < n) {
    if (o + 4 > cap) return -1;
    uint8_t c = s[i];
    if (c < 0x80) {
      d[o++] = alower(c);
      i++;
      continue;
    }
    uint32_t w;
    uint32_t r = decode_rune(s, n, i, &w);
    i += w;
    if (r == 0xFFFD && w == 1) {
      d[o++] = 0xEF; d[o++] = 0xBF; d[o++] = 0xBD;
    } else {
      o += encode_rune(lower_rune(P, r), d + o);
    }
  }
  return o;
}

// ModSecurity urldecode_nonstrict (t:urlDecode)
template <class S, class D>
GI_HD int64_t t_urldecode(S s, uint32_t n, D d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c == '%') {
      if (i + 2 < n && ishex(s[i + 1]) && ishex(s[i + 2])) {
        d[o++] = x2c(s[i + 1], s[i + 2]);
        i += 3;
      } else {
        d[o++] = c;
        i++;
      }
    } else {
      d[o++] = c == '+' ? ' ' : c;
      i++;
    }
  }
  return o;
}

// ModSecurity urldecode_uni_nonstrict (t:urlDecodeUni; %uXXXX low byte, full-width +0x20)
template <class S, class D>
GI_HD int64_t t_urldecodeuni(S s, uint32_t n, D d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c == '%') {
      if (i + 1 < n && (s[i + 1] == 'u' || s[i + 1] == 'U')) {
        if (i + 5 < n && ishex(s[i + 2]) && ishex(s[i + 3]) && ishex(s[i + 4]) && ishex(s[i + 5])) {
          uint8_t b = x2c(s[i + 4], s[i + 5]);
          if (b > 0 && b < 0x5F && (s[i + 2] | 0x20) == 'f' && (s[i + 3] | 0x20) == 'f') b += 0x20;
          d[o++] = b;
          i += 6;
        } else {
          d[o++] = s[i];
          d[o++] = s[i + 1];
          i += 2;
        }
      } else if (i + 2 < n && ishex(s[i + 1]) && ishex(s[i + 2])) {
        d[o++] = x2c(s[i + 1], s[i + 2]);
        i += 3;
      } else {
        d[o++] = c;
        i++;
      }
    } else {
      d[o++] = c == '+' ? ' ' : c;
      i++;
    }
  }
  return o;
}

// strtol(digits, base) & 0xFF, saturating like strtol/ParseInt on overflow
template <class S>
GI_HD uint8_t strtol_byte(S s, uint32_t n, uint32_t base) {
  uint64_t acc = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t v = base == 16 ? hexv(s[i]) : (uint32_t)(s[i] - '0');
    if (acc > ((uint64_t)INT64_MAX - v) / base) return 0xFF;
    acc = acc * base + v;
  }
  return (uint8_t)(acc & 0xFF);
}

// ModSecurity html_entities_decode_inplace (t:htmlEntityDecode)
template <class S, class D>
GI_HD int64_t t_htmlentitydecode(S s, uint32_t n, D d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    uint32_t copy = 1;
    if (s[i] == '&' && i + 1 < n) {
      uint32_t j = i + 1;
      if (s[j] == '#') {
        copy++;
        if (j + 1 < n) {
          j++;
          if (s[j] == 'x' || s[j] == 'X') {
            copy++;
            if (j + 1 < n) {
              j++;
              uint32_t k = j;
              while (j < n && ishex(s[j])) j++;
              if (j > k) {
                d[o++] = strtol_byte(s + k, j - k, 16);
                i = (j < n && s[j] == ';') ? j + 1 : j;
                continue;
              }
            }
          } else {
            uint32_t k = j;
            while (j < n && s[j] >= '0' && s[j] <= '9') j++;
            if (j > k) {
              d[o++] = strtol_byte(s + k, j - k, 10);
              i = (j < n && s[j] == ';') ? j + 1 : j;
              continue;
            }
          }
        }
      } else {
        uint32_t k = j;
        while (j < n && isalnum_(s[j])) j++;
        if (j > k) {
          uint32_t len = j - k;
          int ent = -1;
          const auto x = s + k;
          if (len == 4 && alower(x[0]) == 'q' && alower(x[1]) == 'u' && alower(x[2]) == 'o' && alower(x[3]) == 't') ent = '"';
          else if (len == 3 && alower(x[0]) == 'a' && alower(x[1]) == 'm' && alower(x[2]) == 'p') ent = '&';
          else if (len == 2 && alower(x[0]) == 'l' && alower(x[1]) == 't') ent = '<';
          else if (len == 2 && alower(x[0]) == 'g' && alower(x[1]) == 't') ent = '>';
          else if (len == 4 && alower(x[0]) == 'n' && alower(x[1]) == 'b' && alower(x[2]) == 's' && alower(x[3]) == 'p') ent = 0xA0;
          if (ent >= 0) {
            d[o++] = (uint8_t)ent;
            i = (j < n && s[j] == ';') ? j + 1 : j;
            continue;
          }
          copy = len + 1;
        }
      }
    }
    for (uint32_t z = 0; z < copy && i < n; z++) d[o++] = s[i++];
  }
  return o;
}

GI_HD inline bool ws_or_nbsp(uint8_t c) { return isws(c) || c == 0xA0; }

template <class S, class D>
GI_HD int64_t t_simple(uint8_t code, S s, uint32_t n, D d, uint32_t cap) {
  if (n + 1 > cap) return -1;
  uint32_t o = 0;
  switch (code) {
    case T_REMOVENULLS:
      for (uint32_t i = 0; i < n; i++)
        if (s[i]) d[o++] = s[i];
      return o;
    case T_REPLACENULLS:
      for (uint32_t i = 0; i < n; i++) d[o++] = s[i] ? s[i] : ' ';
      return o;
    case T_REMOVEWHITESPACE:
      for (uint32_t i = 0; i < n; i++)
        if (!ws_or_nbsp(s[i])) d[o++] = s[i];
      return o;
    case T_COMPRESSWHITESPACE: {
      bool inws = false;
      for (uint32_t i = 0; i < n; i++) {
        if (ws_or_nbsp(s[i])) {
          if (!inws) d[o++] = ' ';
          inws = true;
        } else {
          inws = false;
          d[o++] = s[i];
        }
      }
      return o;
    }
    case T_REPLACECOMMENTS: {
      bool inc = false;
      uint32_t i = 0;
      while (i < n) {
        if (!inc) {
          if (s[i] == '/' && i + 1 < n && s[i + 1] == '*') {
            inc = true;
            i += 2;
          } else {
            d[o++] = s[i++];
          }
        } else {
          if (s[i] == '*' && i + 1 < n && s[i + 1] == '/') {
            inc = false;
            i += 2;
            d[o++] = ' ';
          } else {
            i++;
          }
        }
      }
      if (inc) d[o++] = ' ';
      return o;
    }
    case T_CMDLINE: {
      bool space = false;
      for (uint32_t i = 0; i < n; i++) {
        uint8_t c = s[i];
        if (c == '"' || c == '\'' || c == '\\' || c == '^') continue;
        if (c == ' ' || c == ',' || c == ';' || c == '\t' || c == '\r' || c == '\n') {
          if (!space) {
            d[o++] = ' ';
            space = true;
          }
          continue;
        }
        if (c == '/' || c == '(') {
          if (space) {
            o--;
            space = false;
          }
          d[o++] = c;
          continue;
        }
        d[o++] = alower(c);
        space = false;
      }
      return o;
    }
  }
  return -1;
}

// Go unicode.IsSpace
GI_HD inline bool go_isspace(uint32_t r) {
  if (r <= 0xFF) return r == ' ' || (r >= 9 && r <= 13) || r == 0x85 || r == 0xA0;
  return r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 || r == 0x202F ||
         r == 0x205F || r == 0x3000;
}

// Go strings.TrimLeft/TrimRight(unicode.IsSpace)
GI_HD int64_t t_trim(uint8_t code, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  uint32_t a = 0, e = n;
  if (code == T_TRIM || code == T_TRIMLEFT) {
    while (a < e) {
      uint32_t w;
      uint32_t r = decode_rune(s, e, a, &w);
      if ((r == 0xFFFD && w == 1) || !go_isspace(r)) break;
      a += w;
    }
  }
  if (code == T_TRIM || code == T_TRIMRIGHT) {
    while (e > a) {
      uint32_t r, w = 1;
      uint32_t st = e - 1;
      if (s[st] < 0x80) {
        r = s[st];
      } else {
        int64_t k = (int64_t)e - 2;
        int64_t lim = (int64_t)e - 4;
        if (lim < 0) lim = 0;
        bool found = false;
        for (; k >= lim; k--)
          if ((s[k] & 0xC0) != 0x80) { found = true; break; }
        r = 0xFFFD;
        if (found && (uint32_t)k >= a) {
          uint32_t ww;
          uint32_t rr = decode_rune(s, e, (uint32_t)k, &ww);
          if ((uint32_t)k + ww == e && !(rr == 0xFFFD && ww == 1)) {
            r = rr;
            w = ww;
            st = (uint32_t)k;
          }
        }
      }
      if (r == 0xFFFD || !go_isspace(r)) break;
      e = st;
      (void)w;
    }
  }
  if (e - a > cap) return -1;
  for (uint32_t i = a; i < e; i++) d[i - a] = s[i];
  return e - a;
}

// Go path.Clean + coraza normalisePath wrapper
GI_HD int64_t t_normpath(bool win, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (n == 0) return 0;
  if (n + 2 > cap) return -1;
  // work on a '\\' -> '/' view for Win
  auto at = [&](uint32_t i) -> uint8_t { uint8_t c = s[i]; return (win && c == '\\') ? '/' : c; };
  bool rooted = at(0) == '/';
  uint32_t w = 0, r = 0, dotdot = 0;
  if (rooted) {
    d[w++] = '/';
    r = 1;
    dotdot = 1;
  }
  while (r < n) {
    if (at(r) == '/') {
      r++;
    } else if (at(r) == '.' && (r + 1 == n || at(r + 1) == '/')) {
      r++;
    } else if (at(r) == '.' && at(r + 1) == '.' && (r + 2 == n || at(r + 2) == '/')) {
      r += 2;
      if (w > dotdot) {
        w--;
        while (w > dotdot && d[w] != '/') w--;
      } else if (!rooted) {
        if (w > 0) d[w++] = '/';
        d[w++] = '.';
        d[w++] = '.';
        dotdot = w;
      }
    } else {
      if ((rooted && w != 1) || (!rooted && w != 0)) d[w++] = '/';
      while (r < n && at(r) != '/') d[w++] = at(r++);
    }
  }
  if (w == 0) {
    // Clean == "." -> ""
    return 0;
  }
  if (at(n - 1) == '/') d[w++] = '/';
  return w;
}

GI_HD inline bool isodigit(uint8_t c) { return c >= '0' && c <= '7'; }

// ModSecurity js_decode_nonstrict_inplace (t:jsDecode)
template <class S, class D>
GI_HD int64_t t_jsdecode(S s, uint32_t n, D d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    if (s[i] == '\\') {
      if (i + 5 < n && s[i + 1] == 'u' && ishex(s[i + 2]) && ishex(s[i + 3]) && ishex(s[i + 4]) && ishex(s[i + 5])) {
        uint8_t b = x2c(s[i + 4], s[i + 5]);
        if (b > 0 && b < 0x5F && (s[i + 2] | 0x20) == 'f' && (s[i + 3] | 0x20) == 'f') b += 0x20;
        d[o++] = b;
        i += 6;
      } else if (i + 3 < n && s[i + 1] == 'x' && ishex(s[i + 2]) && ishex(s[i + 3])) {
        d[o++] = x2c(s[i + 2], s[i + 3]);
        i += 4;
      } else if (i + 1 < n && isodigit(s[i + 1])) {
        uint32_t j = 0;
        uint8_t buf[3];
        while (i + 1 + j < n && j < 3) {
          buf[j] = s[i + 1 + j];
          j++;
          if (!(i + 1 + j < n && isodigit(s[i + 1 + j]))) break;
        }
        if (j == 3 && buf[0] > '3') j = 2;
        uint32_t v = 0;
        for (uint32_t k = 0; k < j; k++) v = v * 8 + (buf[k] - '0');
        d[o++] = (uint8_t)v;
        i += 1 + j;
      } else if (i + 1 < n) {
        uint8_t c = s[i + 1];
        switch (c) {
          case 'a': c = 7; break;
          case 'b': c = 8; break;
          case 'f': c = 12; break;
          case 'n': c = 10; break;
          case 'r': c = 13; break;
          case 't': c = 9; break;
          case 'v': c = 11; break;
        }
        d[o++] = c;
        i += 2;
      } else {
        while (i < n) d[o++] = s[i++];
      }
    } else {
      d[o++] = s[i++];
    }
  }
  return o;
}

// t:utf8toUnicode: valid multi-byte UTF-8 -> %uXXXX (lowercase hex, >= 4
// digits); ASCII and invalid bytes copied.  [upstream utf8toUnicode.go]
template <class S, class D>
GI_HD int64_t t_utf8tounicode(S s, uint32_t n, D d, uint32_t cap) {
  uint32_t o = 0, i = 0;
  const char* hx = "0123456789abcdef";
  while (i < n) {
    if (o + 8 > cap) return -1;
    uint8_t c = s[i];
    if (c < 0x80) {
      d[o++] = c;
      i++;
      continue;
    }
    uint32_t w;
    uint32_t r = decode_rune(s, n, i, &w);
    if (r == 0xFFFD && w == 1) {
      d[o++] = c;
      i++;
      continue;
    }
    d[o++] = '%';
    d[o++] = 'u';
    int nd = r > 0xFFFFF ? 6 : r > 0xFFFF ? 5 : 4;
    for (int k = nd - 1; k >= 0; k--) d[o++] = hx[(r >> (4 * k)) & 15];
    i += w;
  }
  return o;
}

// ------------------------------------------------ out-of-line transforms
// Decoders / encoders / digests [upstream internal/transformations/
// base64decode.go, base64decodeext.go, base64encode.go, hexdecode.go,
// hexencode.go, sha1.go, md5.go, urlencode.go, cssdecode.go,
// escapeseqdecode.go, removecommentschar.go; ModSecurity ports].  Kept out of
// line so k_stream's inlined LDS chains do not carry their code.

GI_HD inline int b64_val(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// ext = false: base64decode (CR/LF skipped, stop at the first other byte
// outside the alphabet); ext = true: base64decodeext (every such byte skipped)
GI_HD int64_t t_b64decode(bool ext, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, x = 0, k = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    const int v = b64_val(c);
    if (v < 0) {
      if (ext || c == '\r' || c == '\n') continue;
      break;
    }
    x = (x << 6) | (uint32_t)v;
    if (++k == 4) {
      d[o++] = (uint8_t)(x >> 16);
      d[o++] = (uint8_t)(x >> 8);
      d[o++] = (uint8_t)x;
      x = k = 0;
    }
  }
  if (k == 2) {
    d[o++] = (uint8_t)((x << 12) >> 16);
  } else if (k == 3) {
    x <<= 6;
    d[o++] = (uint8_t)(x >> 16);
    d[o++] = (uint8_t)(x >> 8);
  }
  return o;
}

template <class S, class D>
GI_HD int64_t t_b64encode(S s, uint32_t n, D d, uint32_t cap) {
  const char* al = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  const uint64_t out = 4ull * ((n + 2) / 3);
  if (out > cap) return -1;
  uint32_t o = 0, i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t x = ((uint32_t)s[i] << 16) | ((uint32_t)s[i + 1] << 8) | s[i + 2];
    d[o++] = al[x >> 18]; d[o++] = al[(x >> 12) & 63]; d[o++] = al[(x >> 6) & 63]; d[o++] = al[x & 63];
  }
  if (n - i == 1) {
    const uint32_t x = (uint32_t)s[i] << 16;
    d[o++] = al[x >> 18]; d[o++] = al[(x >> 12) & 63]; d[o++] = '='; d[o++] = '=';
  } else if (n - i == 2) {
    const uint32_t x = ((uint32_t)s[i] << 16) | ((uint32_t)s[i + 1] << 8);
    d[o++] = al[x >> 18]; d[o++] = al[(x >> 12) & 63]; d[o++] = al[(x >> 6) & 63]; d[o++] = '=';
  }
  return o;
}

// hex.DecodeString; an error (odd length, non-hex byte) keeps the value
// (rule.go executeTransformations skips a failed transformation)
GI_HD int64_t t_hexdecode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (n > cap) return -1;
  bool ok = (n & 1) == 0;
  for (uint32_t i = 0; i < n && ok; i++) ok = ishex(s[i]);
  if (!ok) {
    for (uint32_t i = 0; i < n; i++) d[i] = s[i];
    return n;
  }
  for (uint32_t i = 0; i < n; i += 2) d[i / 2] = x2c(s[i], s[i + 1]);
  return n / 2;
}

template <class S, class D>
GI_HD int64_t t_hexencode(S s, uint32_t n, D d, uint32_t cap) {
  if (2ull * n > cap) return -1;
  const char* hx = "0123456789abcdef";
  for (uint32_t i = 0; i < n; i++) {
    d[2 * i] = hx[s[i] >> 4];
    d[2 * i + 1] = hx[s[i] & 15];
  }
  return 2 * n;
}

template <class S, class D>
GI_HD int64_t t_urlencode(S s, uint32_t n, D d, uint32_t cap) {
  const char* hx = "0123456789abcdef";
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (o + 3 > cap) return -1;
    const uint8_t c = s[i];
    if (c == ' ') {
      d[o++] = '+';
    } else if (c == '*' || isalnum_(c)) {
      d[o++] = c;
    } else {
      d[o++] = '%';
      d[o++] = hx[c >> 4];
      d[o++] = hx[c & 15];
    }
  }
  return o;
}

GI_HD inline bool c_isspace(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

// ModSecurity css_decode_inplace
template <class S, class D>
GI_HD int64_t t_cssdecode(S s, uint32_t n, D d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    if (s[i] != '\\') {
      d[o++] = s[i++];
      continue;
    }
    if (i + 1 >= n) {  // trailing backslash: dropped
      i++;
      continue;
    }
    i++;
    uint32_t j = 0;
    while (j < 6 && i + j < n && ishex(s[i + j])) j++;
    if (j == 0) {
      if (s[i] != '\n') d[o++] = s[i];
      i++;
      continue;
    }
    uint8_t v;
    if (j == 1) {
      v = hexv(s[i]);
    } else {
      v = x2c(s[i + j - 2], s[i + j - 1]);
      const bool full = j == 4 || (j == 5 && s[i] == '0') || (j == 6 && s[i] == '0' && s[i + 1] == '0');
      if (full && v > 0 && v < 0x5F && (s[i + j - 3] | 0x20) == 'f' && (s[i + j - 4] | 0x20) == 'f') v += 0x20;
    }
    d[o++] = v;
    if (i + j < n && c_isspace(s[i + j])) j++;
    i += j;
  }
  return o;
}

// ModSecurity ansi_c_sequences_decode_inplace
GI_HD int64_t t_escapeseqdecode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    if (s[i] != '\\' || i + 1 >= n) {
      d[o++] = s[i++];
      continue;
    }
    const uint8_t e = s[i + 1];
    int c = -1;
    switch (e) {
      case 'a': c = 7; break;
      case 'b': c = 8; break;
      case 'f': c = 12; break;
      case 'n': c = 10; break;
      case 'r': c = 13; break;
      case 't': c = 9; break;
      case 'v': c = 11; break;
      case '\\': case '?': case '\'': case '"': c = e; break;
    }
    if (c >= 0) {
      d[o++] = (uint8_t)c;
      i += 2;
      continue;
    }
    if (e == 'x' || e == 'X') {
      if (i + 3 < n && ishex(s[i + 2]) && ishex(s[i + 3])) {
        d[o++] = x2c(s[i + 2], s[i + 3]);
        i += 4;
        continue;
      }
    } else if (isodigit(e)) {
      uint32_t j = 0, v = 0;
      while (i + 1 + j < n && j < 3) {
        v = v * 8 + (s[i + 1 + j] - '0');
        j++;
        if (!(i + 1 + j < n && isodigit(s[i + 1 + j]))) break;
      }
      d[o++] = (uint8_t)v;
      i += 1 + j;
      continue;
    }
    d[o++] = e;  // unrecognised escape: the escaped byte
    i += 2;
  }
  return o;
}

// ModSecurity remove_comments_char
GI_HD int64_t t_removecommentschar(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (n > cap) return -1;
  uint32_t o = 0, i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    const uint8_t c1 = i + 1 < n ? s[i + 1] : 0;
    if ((c == '/' && c1 == '*') || (c == '*' && c1 == '/')) {
      i += 2;
    } else if (c == '<' && c1 == '!' && i + 3 < n && s[i + 2] == '-' && s[i + 3] == '-') {
      i += 4;
    } else if (c == '-' && c1 == '-' && i + 2 < n && s[i + 2] == '>') {
      i += 3;
    } else if (c == '-' && c1 == '-') {
      i += 2;
    } else if (c == '#') {
      i += 1;
    } else {
      d[o++] = c;
      i++;
    }
  }
  return o;
}

// Message padding shared by SHA-1 (big-endian length) and MD5 (little-endian):
// 64-byte block b of the padded message s (n bytes).
GI_HD inline void digest_block(const uint8_t* s, uint32_t n, uint32_t b, bool be, uint32_t* w) {
  uint8_t blk[64];
  const uint64_t bits = (uint64_t)n * 8;
  const uint32_t nb = (n + 9 + 63) / 64;
  for (uint32_t k = 0; k < 64; k++) {
    const uint32_t at = b * 64 + k;
    uint8_t v = at < n ? s[at] : at == n ? 0x80 : 0;
    if (b == nb - 1 && k >= 56) v = be ? (uint8_t)(bits >> (8 * (63 - k))) : (uint8_t)(bits >> (8 * (k - 56)));
    blk[k] = v;
  }
  for (uint32_t k = 0; k < 16; k++)
    w[k] = be ? ((uint32_t)blk[4 * k] << 24) | ((uint32_t)blk[4 * k + 1] << 16) | ((uint32_t)blk[4 * k + 2] << 8) | blk[4 * k + 3]
              : ((uint32_t)blk[4 * k + 3] << 24) | ((uint32_t)blk[4 * k + 2] << 16) | ((uint32_t)blk[4 * k + 1] << 8) | blk[4 * k];
}

GI_HD inline uint32_t rotl(uint32_t x, uint32_t c) { return (x << c) | (x >> (32 - c)); }

GI_HD int64_t t_sha1(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (cap < 20) return -1;
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  const uint32_t nb = (n + 9 + 63) / 64;
  for (uint32_t b = 0; b < nb; b++) {
    uint32_t w[16];
    digest_block(s, n, b, true, w);
    uint32_t a = h[0], bb = h[1], c = h[2], dd = h[3], e = h[4];
    for (uint32_t t = 0; t < 80; t++) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        wt = rotl(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
        w[t & 15] = wt;
      }
      uint32_t f, k;
      if (t < 20) { f = (bb & c) | (~bb & dd); k = 0x5A827999u; }
      else if (t < 40) { f = bb ^ c ^ dd; k = 0x6ED9EBA1u; }
      else if (t < 60) { f = (bb & c) | (bb & dd) | (c & dd); k = 0x8F1BBCDCu; }
      else { f = bb ^ c ^ dd; k = 0xCA62C1D6u; }
      const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
      e = dd; dd = c; c = rotl(bb, 30); bb = a; a = tmp;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += dd; h[4] += e;
  }
  for (uint32_t k = 0; k < 5; k++) {
    d[4 * k] = (uint8_t)(h[k] >> 24); d[4 * k + 1] = (uint8_t)(h[k] >> 16);
    d[4 * k + 2] = (uint8_t)(h[k] >> 8); d[4 * k + 3] = (uint8_t)h[k];
  }
  return 20;
}

GI_TABLE uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
GI_TABLE uint8_t kMd5S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};

GI_HD int64_t t_md5(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  if (cap < 16) return -1;
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  const uint32_t nb = (n + 9 + 63) / 64;
  for (uint32_t b = 0; b < nb; b++) {
    uint32_t w[16];
    digest_block(s, n, b, false, w);
    uint32_t a = h[0], bb = h[1], c = h[2], dd = h[3];
    for (uint32_t i = 0; i < 64; i++) {
      uint32_t f, g;
      if (i < 16) { f = (bb & c) | (~bb & dd); g = i; }
      else if (i < 32) { f = (dd & bb) | (~dd & c); g = (5 * i + 1) & 15; }
      else if (i < 48) { f = bb ^ c ^ dd; g = (3 * i + 5) & 15; }
      else { f = c ^ (bb | ~dd); g = (7 * i) & 15; }
      const uint32_t tmp = dd;
      dd = c;
      c = bb;
      bb = bb + rotl(a + f + kMd5K[i] + w[g], kMd5S[(i >> 4) * 4 + (i & 3)]);
      a = tmp;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += dd;
  }
  for (uint32_t k = 0; k < 4; k++) {
    d[4 * k] = (uint8_t)h[k]; d[4 * k + 1] = (uint8_t)(h[k] >> 8);
    d[4 * k + 2] = (uint8_t)(h[k] >> 16); d[4 * k + 3] = (uint8_t)(h[k] >> 24);
  }
  return 16;
}

GI_HD __noinline__ int64_t t_ext(uint8_t code, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  switch (code) {
    case T_BASE64DECODE: return t_b64decode(false, s, n, d, cap);
    case T_BASE64DECODEEXT: return t_b64decode(true, s, n, d, cap);
    case T_BASE64ENCODE: return t_b64encode(s, n, d, cap);
    case T_HEXDECODE: return t_hexdecode(s, n, d, cap);
    case T_HEXENCODE: return t_hexencode(s, n, d, cap);
    case T_SHA1: return t_sha1(s, n, d, cap);
    case T_MD5: return t_md5(s, n, d, cap);
    case T_URLENCODE: return t_urlencode(s, n, d, cap);
    case T_CSSDECODE: return t_cssdecode(s, n, d, cap);
    case T_ESCAPESEQDECODE: return t_escapeseqdecode(s, n, d, cap);
    case T_REMOVECOMMENTSCHAR: return t_removecommentschar(s, n, d, cap);
  }
  return -1;
}

GI_HD __forceinline__ int64_t apply_transform_inl(const DProgram& P, uint8_t code, const uint8_t* s, uint32_t n,
                                                      uint8_t* d, uint32_t cap) {
  switch (code) {
    case T_UTF8TOUNICODE: return t_utf8tounicode(s, n, d, cap);
    case T_LOWERCASE: return t_lowercase(P, s, n, d, cap);
    case T_URLDECODE: return t_urldecode(s, n, d, cap);
    case T_URLDECODEUNI: return t_urldecodeuni(s, n, d, cap);
    case T_HTMLENTITYDECODE: return t_htmlentitydecode(s, n, d, cap);
    case T_LENGTH: return cap < 24 ? -1 : go_itoa((int64_t)n, d);
    case T_TRIM:
    case T_TRIMLEFT:
    case T_TRIMRIGHT: return t_trim(code, s, n, d, cap);
    case T_NORMALIZEPATH: return t_normpath(false, s, n, d, cap);
    case T_NORMALIZEPATHWIN: return t_normpath(true, s, n, d, cap);
    case T_JSDECODE: return t_jsdecode(s, n, d, cap);
    default: return code >= T_BASE64DECODE ? t_ext(code, s, n, d, cap) : t_simple(code, s, n, d, cap);
  }
}

// The chunkable transformations (t_chunkable) over k_body's LDS tiles: the
// pointers are LDS-typed (gi_lds_u8), so every access of the instantiated
// transformations is a ds_* op -- inlined or not (GI_TILE_NOINLINE builds it
// out of line, the A/B check of tests/test_body_chunks.py).
#ifdef GI_TILE_NOINLINE
#define GI_TILE_INL __noinline__
#else
#define GI_TILE_INL __forceinline__
#endif
__device__ GI_TILE_INL int64_t apply_transform_tile(const DProgram& P, uint8_t code, const gi_lds_u8* s, uint32_t n,
                                                    gi_lds_u8* d, uint32_t cap) {
  switch (code) {
    case T_UTF8TOUNICODE: return t_utf8tounicode(s, n, d, cap);
    case T_LOWERCASE: return t_lowercase(P, s, n, d, cap);
    case T_URLDECODE: return t_urldecode(s, n, d, cap);
    case T_URLDECODEUNI: return t_urldecodeuni(s, n, d, cap);
    case T_HTMLENTITYDECODE: return t_htmlentitydecode(s, n, d, cap);
    case T_JSDECODE: return t_jsdecode(s, n, d, cap);
    case T_CSSDECODE: return t_cssdecode(s, n, d, cap);
    case T_URLENCODE: return t_urlencode(s, n, d, cap);
    case T_HEXENCODE: return t_hexencode(s, n, d, cap);
    case T_BASE64ENCODE: return t_b64encode(s, n, d, cap);
    default: return t_simple(code, s, n, d, cap);  // removeNulls, replaceNulls, (compress|remove)Whitespace, cmdLine
  }
}

// Out-of-line instance (generic pointers): k_eval, HBM buffers.  k_stream's
// LDS path inlines apply_transform_inl so every buffer access is a ds_* op.
GI_HD __noinline__ int64_t apply_transform(const DProgram& P, uint8_t code, const uint8_t* s, uint32_t n,
                                                uint8_t* d, uint32_t cap) {
  return apply_transform_inl(P, code, s, n, d, cap);
}

GI_HD uint32_t value_summary(const uint8_t* s, uint32_t n) {
  uint32_t m = 0;
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const uint32_t x = load_u32u(s + i);
    m |= byte_summary((uint8_t)x) | byte_summary((uint8_t)(x >> 8)) | byte_summary((uint8_t)(x >> 16)) |
         byte_summary((uint8_t)(x >> 24));
  }
  for (; i < n; i++) m |= byte_summary(s[i]);
  return m;
}
// the same through a 256-entry table (k_stream keeps it in LDS)
GI_HD __forceinline__ uint32_t value_summary_lut(const uint16_t* lut, const uint8_t* s, uint32_t n) {
  uint32_t m = 0;
  for (uint32_t i = 0; i < n; i++) m |= lut[s[i]];
  return m;
}
// ------------------------------------------------ matched-variable state
// coraza tx.matchVariable on every operator match: MATCHED_VAR /
// MATCHED_VAR_NAME = the matched (transformed) value and "VAR[:key]";
// MATCHED_VARS(_NAMES) += (name -> value), an existing name (compared ASCII
// case-insensitively, the collection's key rule) keeping its position with
// the new value.  Only kept when the program reads it (DProgram.mv_used); all
// strings are copied (the matched value may sit in a transformation buffer).
// Area layout: [MvState 64 B][MvEnt x cap_e][arena cap_a][MATCHED_VAR cap_v][MATCHED_VAR_NAME cap_n]
struct MvEnt {
  const uint8_t* name;
  const uint8_t* v;
  uint32_t nn, vn;
  uint64_t _pad;
};
struct MvState {
  uint32_t n, cap_e;       // MATCHED_VARS entries of the current top-level rule
  uint32_t nb, cap_a;      // arena bytes used (reset with the entries)
  uint32_t cap_v, cap_n;
  uint32_t cur_vn, cur_nn; // MATCHED_VAR / MATCHED_VAR_NAME lengths (persist across rules)
  uint32_t keep;           // the current rule's chain reads MATCHED_VARS(_NAMES): record the entries (RF2_MVS)
  uint32_t cur;            // MATCHED_VAR(_NAME) of the current rule's matches can be read (RF2_MVCUR)
  uint32_t _pad[6];
};
static_assert(sizeof(MvState) == 64 && sizeof(MvEnt) == 32, "MvState layout");

GI_HD inline MvEnt* mv_ents(MvState* m) { return (MvEnt*)(m + 1); }
GI_HD inline uint8_t* mv_arena(MvState* m) { return (uint8_t*)(mv_ents(m) + m->cap_e); }
GI_HD inline uint8_t* mv_curval(MvState* m) { return mv_arena(m) + ((m->cap_a + 15) & ~15u); }
GI_HD inline uint8_t* mv_curname(MvState* m) { return mv_curval(m) + ((m->cap_v + 15) & ~15u); }

// The variable's name as a rule writes it (coraza RuleVariable.Name()).
GI_HD const char* var_name(uint32_t var) {
  switch (var) {
    case S_REQUEST_METHOD: return "REQUEST_METHOD";
    case S_REQUEST_PROTOCOL: return "REQUEST_PROTOCOL";
    case S_REQUEST_URI: return "REQUEST_URI";
    case S_REQUEST_URI_RAW: return "REQUEST_URI_RAW";
    case S_REQUEST_LINE: return "REQUEST_LINE";
    case S_REQUEST_FILENAME: return "REQUEST_FILENAME";
    case S_REQUEST_BASENAME: return "REQUEST_BASENAME";
    case S_QUERY_STRING: return "QUERY_STRING";
    case S_REQUEST_BODY: return "REQUEST_BODY";
    case S_REQUEST_BODY_LENGTH: return "REQUEST_BODY_LENGTH";
    case S_REQBODY_ERROR: return "REQBODY_ERROR";
    case S_REQBODY_ERROR_MSG: return "REQBODY_ERROR_MSG";
    case S_REQBODY_PROCESSOR: return "REQBODY_PROCESSOR";
    case S_MULTIPART_STRICT_ERROR: return "MULTIPART_STRICT_ERROR";
    case S_REMOTE_ADDR: return "REMOTE_ADDR";
    case S_SERVER_NAME: return "SERVER_NAME";
    case S_REMOTE_PORT: return "REMOTE_PORT";
    case S_FILES_COMBINED_SIZE: return "FILES_COMBINED_SIZE";
    case S_ARGS_COMBINED_SIZE: return "ARGS_COMBINED_SIZE";
    case S_FULL_REQUEST_LENGTH: return "FULL_REQUEST_LENGTH";
    case S_URLENCODED_ERROR: return "URLENCODED_ERROR";
    case S_INBOUND_DATA_ERROR: return "INBOUND_DATA_ERROR";
    case V_ARGS_GET: return "ARGS_GET";
    case V_ARGS_POST: return "ARGS_POST";
    case V_ARGS: return "ARGS";
    case V_REQUEST_HEADERS: return "REQUEST_HEADERS";
    case V_REQUEST_COOKIES: return "REQUEST_COOKIES";
    case V_TX: return "TX";
    case V_ARGS_GET_NAMES: return "ARGS_GET_NAMES";
    case V_ARGS_POST_NAMES: return "ARGS_POST_NAMES";
    case V_ARGS_NAMES: return "ARGS_NAMES";
    case V_REQUEST_HEADERS_NAMES: return "REQUEST_HEADERS_NAMES";
    case V_REQUEST_COOKIES_NAMES: return "REQUEST_COOKIES_NAMES";
    case V_XML: return "XML";
    case V_FILES: return "FILES";
    case V_FILES_NAMES: return "FILES_NAMES";
    case V_FILES_SIZES: return "FILES_SIZES";
    case V_FILES_TMPNAMES: return "FILES_TMPNAMES";
    case V_MULTIPART_PART_HEADERS: return "MULTIPART_PART_HEADERS";
    case V_MATCHED_VAR: return "MATCHED_VAR";
    case V_MATCHED_VAR_NAME: return "MATCHED_VAR_NAME";
    case V_MATCHED_VARS: return "MATCHED_VARS";
    case V_MATCHED_VARS_NAMES: return "MATCHED_VARS_NAMES";
  }
  return "";
}

// tx.matchVariable; false when a capacity is exceeded (the request is flagged).
GI_HD __noinline__ bool mv_record(MvState* m, uint32_t var, const uint8_t* k, uint32_t kn, const uint8_t* v,
                                       uint32_t vn) {
  if (!m->cur && !m->keep) return true;  // nothing can read what this match sets
  const char* vnm = var_name(var);
  uint32_t vl = 0;
  while (vnm[vl]) vl++;
  const uint32_t nn = vl + (kn ? 1 + kn : 0);
  if (vn > m->cap_v || nn > m->cap_n) return false;
  // MATCHED_VAR_NAME / MATCHED_VAR
  uint8_t* cn = mv_curname(m);
  for (uint32_t i = 0; i < vl; i++) cn[i] = (uint8_t)vnm[i];
  if (kn) {
    cn[vl] = ':';
    copy_bytes(cn + vl + 1, k, kn);
  }
  m->cur_nn = nn;
  uint8_t* cv = mv_curval(m);
  copy_bytes(cv, v, vn);
  m->cur_vn = vn;
  if (!m->keep) return true;  // nothing reads this rule's MATCHED_VARS
  // MATCHED_VARS SetIndex(name, 0, value)
  MvEnt* e = mv_ents(m);
  uint32_t at = m->n;
  for (uint32_t j = 0; j < m->n; j++)
    if (e[j].nn == nn && eq_ascii_ci_both(e[j].name, cn, nn)) {
      at = j;
      break;
    }
  const uint32_t need = vn + (at == m->n ? nn : 0);
  if (m->nb + need > m->cap_a || (at == m->n && m->n >= m->cap_e)) return false;
  uint8_t* a = mv_arena(m) + m->nb;
  copy_bytes(a, v, vn);
  e[at].v = a;
  e[at].vn = vn;
  if (at == m->n) {
    uint8_t* nm = a + vn;
    copy_bytes(nm, cn, nn);
    e[at].name = nm;
    e[at].nn = nn;
    m->n++;
  } else {  // the key as last written (a case-insensitive equal name has the same length)
    uint8_t* nm = (uint8_t*)e[at].name;
    copy_bytes(nm, cn, nn);
  }
  m->nb += need;
  return true;
}

// ------------------------------------------------------------ transaction
struct Tx {
  const DProgram* P;
  Field* fields;
  uint32_t nf, cap_f;
  Slot* slots;               // TX slot 0 of this request; slot s at slots[s * n_req] (request-major SoA:
                             // the lanes of a wave walk the same rule, so they touch the same slot)
  uint8_t* bytes;
  uint32_t nb, cap_b;
  uint8_t* t0;
  uint8_t* t1;
  uint32_t cap_t;
  uint8_t* mt;
  uint32_t cap_mt;
  uint8_t* txa;
  uint32_t ntx, cap_tx;
  Str* single;               // ReqHdr::single (per-request, in HBM scratch)
  const uint32_t* hits;      // this request's phase-A hit word of slot s at hits[(s / 32) * hstride]
  uint32_t hstride;          // n_req (the batch's hit words in HBM) or 1 (k_eval_wave's LDS copy)
  const uint32_t* vmap;      // the request's phase-A value signatures (word 2f + side: bit slot % 32)
  const uint32_t* hset;      // the request's exact hit set (nullptr: none, or it overflowed)
  uint32_t hmask;
  uint32_t nf_pa;            // fields [0, nf_pa) went through phase A (value map valid)
  uint32_t n_req, req;
  bool has_post;             // ARGS_POST fields phase A did not see (phase-A bits of RF_BODYDEP links void)
  bool body_spec;            // the body went through k_collect's processor: k_body tested REQUEST_BODY
  bool pa_void;              // phase-A arena overflowed: no phase-A bit is trusted
  int64_t (*removed)[2];     // ctl:ruleRemoveById ranges (8, in the request's scratch region)
  struct RmTarget {          // ctl:ruleRemoveTargetById entries (8, after the ranges)
    int64_t lo, hi;
    uint32_t var, koff, klen, _pad;
  }* rtgt;
  uint32_t nrtgt;
  const uint32_t* kx;        // kind index (build_kindex; nullptr: scan all fields)
  uint32_t nremoved;
  uint32_t rm_groups;        // ctl:ruleRemoveByTag / ByMsg groups removed (DProgram.rule_groups)
  uint32_t cur_groups;       // removal groups of the top-level rule being evaluated
  uint8_t allow;             // allow action in effect (D_ALLOW_*; 0: none)
  bool prefix;               // gate stage 1, the request's body processed: stop at the first RF2_BODY_PA rule
  bool prefix_spec;          // ... and its body fields are the speculative parser's (scanned by the prefix streams)
  bool bail;                 // ... and it stopped there (the body stage re-evaluates it)
  uint8_t engine, body_access, body_proc, phase;
  uint8_t force_body;
  int32_t skip_after;
  int32_t skip;
  int32_t int_rule, int_status;
  uint8_t int_action, int_phase;
  bool interrupted;
  uint16_t flags;
  uint32_t nmatched;
  uint32_t* mout;
  uint32_t mcap;
  MvState* mv;               // matched-variable state (nullptr unless DProgram.mv_used)
  uint32_t* capws;           // pike_match workspace (observable captures; nullptr: none)
  bool crec;                 // capture records are written (capws and the batch's record rows)
  bool rcoll;                // the body went through the XML / multipart processor: residual body collections
                             // (RF2_RESID_COLL) may have entries
  bool rbody;                // REQUEST_BODY is not empty (RF2_RESID_RB)
  uint8_t* capbuf;           // per capture group g: cap_t bytes holding TX.g's value
  uint8_t* dyn;              // TX keys macro-key setvars created (DynHdr; nullptr: the program has none)
  uint64_t wm0, wm1;         // TX slots < 128 this request owns (written); the others read the snapshot
  bool snap;                 // the folded prefix ran (phase 1 started): unowned slots read DProgram.tx_snap
  uint32_t cur_id;           // id of the top-level rule being evaluated (capture records)
  bool profon;               // GI_PROF counters (diagnostics)
  uint32_t prof_visits, prof_evals, prof_rules, prof_ops;
  uint64_t prof_eval_cyc, prof_act_cyc;
  unsigned long long* prof_rule_cyc;  // [rule link] cycles (GI_PROF)
};

#define TXS(t, s) ((t).slots[(uint64_t)(s) * (t).n_req])

// TX slot s, copy on write over the folded snapshot (compile.cpp
// fold_program): a slot the request has not written reads the program's
// snapshot (once the folded prefix ran; before, every slot is unset), so no
// per-request TX initialisation touches HBM.  Slots >= 128 are always owned
// (initialised at phase-1 start).
GI_HD __forceinline__ bool tx_owned(const Tx& t, uint32_t s) {
  return s >= 128 || ((s < 64 ? t.wm0 >> s : t.wm1 >> (s - 64)) & 1u);
}
GI_HD __forceinline__ Slot slot_rd(const Tx& t, uint32_t s) {
  if (tx_owned(t, s)) return TXS(t, s);
  if (t.snap) return ((const Slot*)t.P->tx_snap)[s];
  Slot z;
  z.num = 0;
  z.n = 0;
  z.state = 0;
  return z;
}
GI_HD __forceinline__ Slot& slot_wr(Tx& t, uint32_t s) {
  if (!tx_owned(t, s)) {
    TXS(t, s) = slot_rd(t, s);
    if (s < 64) t.wm0 |= 1ull << s;
    else t.wm1 |= 1ull << (s - 64);
  }
  return TXS(t, s);
}

// tx_alloc / add_field serve Tx and the body parser's JsonCtx alike
template <class C>
GI_HD inline uint8_t* tx_alloc(C& t, uint32_t n) {
  if (t.nb + n > t.cap_b) {
    t.flags |= GI_REQ_OVERFLOW;
    return nullptr;
  }
  uint8_t* p = t.bytes + t.nb;
  t.nb += n;
  return p;
}

template <class C>
GI_HD inline void add_field(C& t, uint8_t kind, const uint8_t* k, uint32_t kn, const uint8_t* v, uint32_t vn) {
  if (t.nf >= t.cap_f) {
    t.flags |= GI_REQ_OVERFLOW;
    return;
  }
  Field& f = t.fields[t.nf++];
  f.k = k;
  f.v = v;
  f.kn = kn;
  f.vn = vn;
  f.kind = kind;
}

// lenient %XX / '+' decoding (coraza internal/url QueryUnescape)
GI_HD uint32_t query_unescape(const uint8_t* s, uint32_t n, uint8_t* d) {
  uint32_t o = 0, i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c == '%' && i + 2 < n && ishex(s[i + 1]) && ishex(s[i + 2])) {
      d[o++] = x2c(s[i + 1], s[i + 2]);
      i += 3;
    } else {
      d[o++] = c == '+' ? ' ' : c;
      i++;
    }
  }
  return o;
}

// coraza internal/url ParseQuery(query, '&') -> fields of `kind`.  A key or
// value without '%' / '+' is its own decoding: the field points into the
// request bytes, and only escaped parts are decoded into the arena.
GI_HD __forceinline__ void parse_query(Tx& t, const uint8_t* q, uint32_t n, uint8_t kind) {
  uint32_t i = 0;
  while (i < n) {
    uint32_t j = i, e = 0xFFFFFFFFu;
    bool kesc = false, vesc = false;
    for (; j < n; j++) {
      const uint8_t c = q[j];
      if (c == '&') break;
      if (c == '=' && e == 0xFFFFFFFFu) e = j;
      else if (c == '%' || c == '+') (e == 0xFFFFFFFFu ? kesc : vesc) = true;
    }
    if (j > i) {
      if (e == 0xFFFFFFFFu) e = j;
      const uint8_t* k = q + i;
      const uint32_t kn = e - i;
      const uint8_t* v = q + (e < j ? e + 1 : j);
      const uint32_t vn = e < j ? j - e - 1 : 0;
      const uint8_t* dk = k;
      uint32_t dkn = kn;
      const uint8_t* dv = v;
      uint32_t dvn = vn;
      if (kesc || vesc) {
        uint8_t* d = tx_alloc(t, (kesc ? kn : 0) + (vesc ? vn : 0));
        if (!d) return;
        if (kesc) {
          dkn = query_unescape(k, kn, d);
          dk = d;
          d += dkn;
        }
        if (vesc) {
          dvn = query_unescape(v, vn, d);
          dv = d;
        }
      }
      add_field(t, kind, dk, dkn, dv, dvn);
    }
    i = j + 1;
  }
}

// ------------------------------------------------------------ JSON body
// coraza internal/bodyprocessors/json.go (readJSON / readItems over
// tidwall/gjson v1.18.0), restated as one iterative pass per request:
// ARGS_POST "json.<k1>.<k2>..." (object members unescaped, array indices
// decimal), strings unescaped, numbers / true / false raw, null "", and a
// non-empty array's own key = its element count after its elements.  A key
// written twice is one entry (Go map + ARGS_POST SetIndex(key, 0)) at the
// first write's position holding the last write's value.
// Read left to right; the first of these events decides (oracle: json_flatten):
//  * a syntax error (not RFC 8259 JSON: gjson.Valid false) -> GI_REQ_BODY_ERROR:
//    readJSON's error, so the caller sets REQBODY_ERROR and drops ARGS_POST;
//  * an engine limit -> GI_REQ_UNSUPPORTED_BODY: a scalar root value, nesting
//    deeper than GI_JSON_MAX_DEPTH, or flattened keys + unescaped strings +
//    array counts over 4 x body + 1024 bytes (the arena runtime.cpp reserves;
//    deep nesting makes the keys quadratic).
#define GI_JSON_MAX_DEPTH 64

struct JFrame {
  uint32_t koff, kn;  // the container's own key (offset into t.bytes)
  uint32_t count;     // members / elements seen
  uint32_t is_arr;
};

GI_HD inline bool json_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

GI_HD inline uint32_t hex4(const uint8_t* s) {
  return (hexv(s[0]) << 12) | (hexv(s[1]) << 8) | (hexv(s[2]) << 4) | hexv(s[3]);
}

// Validates the string whose opening quote is at s[i]; returns the index
// after the closing quote (0 on error) and whether it holds escapes.
GI_HD uint32_t json_string_end(const uint8_t* s, uint32_t n, uint32_t i, bool* esc) {
  *esc = false;
  i++;
  while (i < n) {
    // four plain bytes at a time (none is '"', '\\' or a control byte: the
    // per-byte step below would only advance over them)
    while (i + 4 <= n) {
      const uint32_t w = load_u32u(s + i);
      const uint32_t q = w ^ 0x22222222u, b = w ^ 0x5C5C5C5Cu;
      if ((((q - 0x01010101u) & ~q) | ((b - 0x01010101u) & ~b) | ((w - 0x20202020u) & ~w)) & 0x80808080u) break;
      i += 4;
    }
    if (i >= n) break;
    const uint8_t c = s[i];
    if (c == '"') return i + 1;
    if (c < 0x20) return 0;
    if (c == '\\') {
      if (i + 1 >= n) return 0;
      const uint8_t e = s[i + 1];
      *esc = true;
      if (e == 'u') {
        if (i + 6 > n || !ishex(s[i + 2]) || !ishex(s[i + 3]) || !ishex(s[i + 4]) || !ishex(s[i + 5])) return 0;
        i += 6;
        continue;
      }
      if (e != '"' && e != '\\' && e != '/' && e != 'b' && e != 'f' && e != 'n' && e != 'r' && e != 't') return 0;
      i += 2;
      continue;
    }
    i++;
  }
  return 0;
}

GI_HD inline uint32_t utf8_put(uint32_t r, uint8_t* d) {
  if ((r >= 0xD800 && r <= 0xDFFF) || r > 0x10FFFF) r = 0xFFFD;
  if (r < 0x80) { d[0] = (uint8_t)r; return 1; }
  if (r < 0x800) { d[0] = 0xC0 | (r >> 6); d[1] = 0x80 | (r & 0x3F); return 2; }
  if (r < 0x10000) {
    d[0] = 0xE0 | (r >> 12); d[1] = 0x80 | ((r >> 6) & 0x3F); d[2] = 0x80 | (r & 0x3F);
    return 3;
  }
  d[0] = 0xF0 | (r >> 18); d[1] = 0x80 | ((r >> 12) & 0x3F); d[2] = 0x80 | ((r >> 6) & 0x3F); d[3] = 0x80 | (r & 0x3F);
  return 4;
}

// gjson unescape of a validated string body; never longer than its input.
GI_HD uint32_t json_unescape(const uint8_t* s, uint32_t n, uint8_t* d) {
  uint32_t o = 0, i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c != '\\') {
      d[o++] = c;
      i++;
      continue;
    }
    const uint8_t e = s[i + 1];
    if (e != 'u') {
      d[o++] = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
      i += 2;
      continue;
    }
    uint32_t r = hex4(s + i + 2);
    i += 6;
    if (r >= 0xD800 && r < 0xE000) {  // utf16.IsSurrogate: consume a following \uXXXX
      if (n - i >= 6 && s[i] == '\\' && s[i + 1] == 'u') {
        const uint32_t r2 = hex4(s + i + 2);
        i += 6;
        r = (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000) ? 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00) : 0xFFFD;
      } else {
        r = 0xFFFD;
      }
    }
    o += utf8_put(r, d + o);
  }
  return o;
}

// gjson validnumber at s[i]; returns the end index (0 on error).
GI_HD uint32_t json_number_end(const uint8_t* s, uint32_t n, uint32_t i) {
  if (i < n && s[i] == '-') i++;
  if (i >= n || s[i] < '0' || s[i] > '9') return 0;
  if (s[i] == '0') {
    i++;
  } else {
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
  }
  if (i < n && s[i] == '.') {
    i++;
    if (i >= n || s[i] < '0' || s[i] > '9') return 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
  }
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    i++;
    if (i < n && (s[i] == '+' || s[i] == '-')) i++;
    if (i >= n || s[i] < '0' || s[i] > '9') return 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
  }
  return i;
}


GI_HD inline bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}

// Fold repeated keys of fields [f0, t.nf) (first position, last value) with
// an open-addressing table in the transform scratch t.t1.
template <class C>
GI_HD __forceinline__ void json_fold_keys(C& t, uint32_t f0) {
  const uint32_t nf = t.nf - f0;
  const uint32_t cap = t.cap_t / 4;  // > body/2 + 2 >= nf (runtime.cpp sizing)
  if (nf < 2) return;
  if (nf >= cap) {
    t.flags |= GI_REQ_OVERFLOW;
    return;
  }
  // the smallest power of two >= 2 nf that the scratch holds (the fold does
  // not depend on the table size; zeroing cap words cost more than the parse)
  uint32_t tsize = 16;
  while (tsize < 2 * nf && 2 * tsize <= cap) tsize *= 2;
  if (tsize > cap || tsize <= nf) tsize = cap;  // (cap > nf: an empty slot always remains)
  const bool pow2 = (tsize & (tsize - 1)) == 0;
  uint32_t* tab = (uint32_t*)t.t1;
  for (uint32_t k = 0; k < tsize; k++) tab[k] = 0;
  bool any = false;
  for (uint32_t i = f0; i < t.nf; i++) {
    Field& f = t.fields[i];
    const uint32_t hv = gi_fnv1a(f.k, f.kn, false);
    uint32_t h = pow2 ? (hv & (tsize - 1)) : hv % tsize;
    while (true) {
      const uint32_t e = tab[h];
      if (e == 0) {
        tab[h] = i + 1;
        break;
      }
      Field& g = t.fields[e - 1];
      if (g.kn == f.kn && bytes_equal(g.k, f.k, f.kn)) {
        g.v = f.v;
        g.vn = f.vn;
        f.kind = 0;  // folded into g
        any = true;
        break;
      }
      h = h + 1 == tsize ? 0 : h + 1;
    }
  }
  if (!any) return;
  uint32_t o = f0;
  for (uint32_t i = f0; i < t.nf; i++)
    if (t.fields[i].kind) t.fields[o++] = t.fields[i];
  t.nf = o;
}

template <class C>
GI_HD __forceinline__ void parse_json_body(C& t, const uint8_t* s, uint32_t n) {
  const uint32_t f0 = t.nf;
  uint32_t i = 0;
  while (i < n && json_ws(s[i])) i++;
  if (i >= n || (s[i] != '{' && s[i] != '[')) {  // (before any allocation: runtime.cpp sizes
    const uint8_t c0 = i < n ? s[i] : 0;          // the parser arena for '{' / '[' bodies only)
    const bool scalar = i < n && (c0 == '"' || c0 == '-' || (c0 >= '0' && c0 <= '9') || c0 == 't' || c0 == 'f' || c0 == 'n');
    t.flags |= scalar ? GI_REQ_UNSUPPORTED_BODY : GI_REQ_BODY_ERROR;
    return;
  }
  JFrame* st = (JFrame*)tx_alloc(t, (GI_JSON_MAX_DEPTH + 1) * sizeof(JFrame) + 8);
  if (!st) return;
  st = (JFrame*)(((uintptr_t)st + 7) & ~(uintptr_t)7);
  uint8_t* root = tx_alloc(t, 4);
  if (!root) return;
  root[0] = 'j'; root[1] = 's'; root[2] = 'o'; root[3] = 'n';
  uint32_t d = 1;
  st[0] = {(uint32_t)(root - t.bytes), 4, 0, s[i] == '[' ? 1u : 0u};
  const uint64_t lim = 4ull * n + 1024;
  uint64_t jb = 0;  // flattened bytes (keys, unescaped strings, counts)
  i++;
  bool bad = false;     // syntax error
  bool limit = false;   // engine limit
  while (d > 0 && !bad && !limit && !(t.flags & GI_REQ_ERROR_MASK)) {
    JFrame& F = st[d - 1];
    while (i < n && json_ws(s[i])) i++;
    if (i >= n) { bad = true; break; }
    if (s[i] == (F.is_arr ? ']' : '}')) {
      i++;
      if (F.is_arr && F.count) {
        uint8_t* nb = tx_alloc(t, 12);
        if (!nb) return;
        const uint32_t dn = go_itoa((int64_t)F.count, nb);
        t.nb -= 12 - dn;
        jb += dn;
        if (jb > lim) { limit = true; break; }
        add_field(t, FK_ARG_POST, t.bytes + F.koff, F.kn, nb, dn);
      }
      d--;
      continue;
    }
    if (F.count) {
      if (s[i] != ',') { bad = true; break; }
      i++;
      while (i < n && json_ws(s[i])) i++;
    }
    // the element's key: parent key + '.' + member name / index
    uint8_t* key;
    uint32_t kn;
    if (F.is_arr) {
      key = tx_alloc(t, F.kn + 12);
      if (!key) return;
      copy_bytes(key, t.bytes + F.koff, F.kn);
      key[F.kn] = '.';
      kn = F.kn + 1 + go_itoa((int64_t)F.count, key + F.kn + 1);
      t.nb -= F.kn + 12 - kn;  // give back the unused tail
      jb += kn;
      if (jb > lim) { limit = true; break; }
    } else {
      if (i >= n || s[i] != '"') { bad = true; break; }
      bool esc;
      const uint32_t e = json_string_end(s, n, i, &esc);
      if (!e) { bad = true; break; }
      const uint32_t rn = e - i - 2;
      key = tx_alloc(t, F.kn + 1 + rn);
      if (!key) return;
      copy_bytes(key, t.bytes + F.koff, F.kn);
      key[F.kn] = '.';
      uint32_t sn = rn;
      if (esc) {
        sn = json_unescape(s + i + 1, rn, key + F.kn + 1);
      } else {
        copy_bytes(key + F.kn + 1, s + i + 1, rn);
      }
      kn = F.kn + 1 + sn;
      t.nb -= rn - sn;
      jb += kn;
      if (jb > lim) { limit = true; break; }
      i = e;
      while (i < n && json_ws(s[i])) i++;
      if (i >= n || s[i] != ':') { bad = true; break; }
      i++;
      while (i < n && json_ws(s[i])) i++;
    }
    F.count++;
    if (i >= n) { bad = true; break; }
    const uint8_t c = s[i];
    if (c == '{' || c == '[') {
      if (d >= GI_JSON_MAX_DEPTH) { limit = true; break; }
      st[d++] = {(uint32_t)(key - t.bytes), kn, 0, c == '[' ? 1u : 0u};
      i++;
    } else if (c == '"') {
      bool esc;
      const uint32_t e = json_string_end(s, n, i, &esc);
      if (!e) { bad = true; break; }
      const uint32_t rn = e - i - 2;
      if (esc) {
        uint8_t* v = tx_alloc(t, rn);
        if (!v && rn) return;
        const uint32_t vn = json_unescape(s + i + 1, rn, v);
        t.nb -= rn - vn;
        jb += vn;
        if (jb > lim) { limit = true; break; }
        add_field(t, FK_ARG_POST, key, kn, v, vn);
      } else {
        add_field(t, FK_ARG_POST, key, kn, s + i + 1, rn);
      }
      i = e;
    } else if (c == 't' || c == 'f' || c == 'n') {
      const uint32_t ln = c == 'f' ? 5 : 4;
      const char* lit = c == 't' ? "true" : c == 'f' ? "false" : "null";
      if (i + ln > n) { bad = true; break; }
      for (uint32_t k = 0; k < ln; k++)
        if (s[i + k] != (uint8_t)lit[k]) bad = true;
      if (bad) break;
      add_field(t, FK_ARG_POST, key, kn, s + i, c == 'n' ? 0 : ln);
      i += ln;
    } else {
      const uint32_t e = json_number_end(s, n, i);
      if (!e) { bad = true; break; }
      add_field(t, FK_ARG_POST, key, kn, s + i, e - i);
      i = e;
    }
  }
  if (!bad && !limit && d == 0) {
    while (i < n && json_ws(s[i])) i++;
    bad = i != n;
  }
  if (limit) {
    t.flags |= GI_REQ_UNSUPPORTED_BODY;
    return;
  }
  if (bad || d != 0) {
    t.flags |= GI_REQ_BODY_ERROR;
    return;
  }
  if (!(t.flags & GI_REQ_ERROR_MASK)) json_fold_keys(t, f0);
}

// The parser state k_eval hands to the out-of-line instance: passing the
// whole Tx by reference would pin it in scratch memory for the entire kernel.
struct JsonCtx {
  Field* fields;
  uint32_t nf, cap_f;
  uint8_t* bytes;
  uint32_t nb, cap_b;
  uint8_t* t1;
  uint32_t cap_t;
  uint16_t flags;
};

GI_HD __noinline__ void parse_json_body_ool(JsonCtx* c, const uint8_t* s, uint32_t n) {
  parse_json_body(*c, s, n);
}

// ------------------------------------------------------------ multipart body
// [upstream coraza internal/bodyprocessors/multipart.go ProcessRequest over
// Go's mime.ParseMediaType, mime/multipart.Reader.NextPart and
// textproto.ReadMIMEHeader], one sequential pass; oracle/multipart.py states
// the same semantics, their limits and the error classes.  Output fields:
// per part, its headers (FK_PART_HEADER: part name, "Key: value", sorted by
// key), then either the file entries (FK_FILE "", file name; FK_FILE_SIZE
// file name, size, SetIndex per name; FK_FILE_NAME "", part name) or the
// field (FK_ARG_POST part name, data -> points into the body).
enum MpErr : uint8_t {
  MP_OK = 0, MP_E_MEDIA, MP_E_NOTMP, MP_E_EMPTYB, MP_E_EOF, MP_E_BUFFULL, MP_E_EXPECT, MP_E_UNEXP, MP_E_HDR,
  MP_E_DATA, MP_E_COUNT
};
// REQBODY_ERROR_MSG per error class ("<processor>: <error>", generateRequestBodyError)
GI_TABLE char kMpErrMsg[MP_E_COUNT][56] = {
    "", "MULTIPART: mime: invalid media type", "MULTIPART: not a multipart body",
    "MULTIPART: multipart: boundary is empty", "MULTIPART: multipart: NextPart: EOF",
    "MULTIPART: multipart: NextPart: bufio: buffer full", "MULTIPART: multipart: expecting a new Part",
    "MULTIPART: multipart: unexpected line in Next()", "MULTIPART: multipart: NextPart: malformed MIME header",
    "MULTIPART: unexpected EOF"};

GI_HD inline bool mp_tspecial(uint8_t c) {
  switch (c) {
    case '(': case ')': case '<': case '>': case '@': case ',': case ';': case ':': case '\\': case '"':
    case '/': case '[': case ']': case '?': case '=':
      return true;
  }
  return false;
}
GI_HD inline bool mp_token(uint8_t c) { return c > 0x20 && c < 0x7F && !mp_tspecial(c); }
GI_HD inline bool mp_lws(uint8_t c) { return c == ' ' || c == '\t'; }

// Next ";key=value" of a media type at v[*i]: 0 ok, 1 no more, -1 syntax error.
GI_HD int mp_next_param(const uint8_t* v, uint32_t n, uint32_t* i, uint32_t* ks, uint32_t* ke, uint32_t* vs,
                             uint32_t* ve, bool* quoted) {
  uint32_t p = *i;
  while (p < n && mp_lws(v[p])) p++;
  if (p >= n) return 1;
  if (v[p] != ';') return -1;
  p++;
  while (p < n && mp_lws(v[p])) p++;
  if (p >= n) return 1;  // trailing ';'
  const uint32_t k0 = p;
  while (p < n && mp_token(v[p])) p++;
  if (p == k0) return -1;
  *ks = k0;
  *ke = p;
  while (p < n && mp_lws(v[p])) p++;
  if (p >= n || v[p] != '=') return -1;
  p++;
  while (p < n && mp_lws(v[p])) p++;
  if (p < n && v[p] == '"') {
    uint32_t q = p + 1;
    while (q < n && v[q] != '"') {
      if (v[q] == '\r' || v[q] == '\n') return -1;
      if (v[q] == '\\' && q + 1 < n && mp_tspecial(v[q + 1])) q++;
      q++;
    }
    if (q >= n) return -1;
    *vs = p + 1;
    *ve = q;
    *quoted = true;
    p = q + 1;
  } else {
    uint32_t q = p;
    while (q < n && mp_token(v[q])) q++;
    if (q == p) return -1;
    *vs = p;
    *ve = q;
    *quoted = false;
    p = q;
  }
  *i = p;
  return 0;
}

// mime.ParseMediaType(v) restricted to what the processor reads: the media
// type [*ts, *te) (not lowercased) and up to two wanted parameters (keys
// lowercase literals; values unescaped into the arena when quoted with
// escapes).  Returns 0 ok, 1 error, 2 unsupported (RFC 2231 parameter).
template <class C>
GI_HD int mp_media(C& t, const uint8_t* v, uint32_t n, uint32_t* ts, uint32_t* te, const char* w0, Str* o0,
                        const char* w1, Str* o1) {
  o0->p = CS_ZERO;
  o0->n = 0;
  if (o1) {
    o1->p = CS_ZERO;
    o1->n = 0;
  }
  uint32_t semi = 0;
  while (semi < n && v[semi] != ';') semi++;
  uint32_t a = 0, b = semi;
  while (a < b && mp_lws(v[a])) a++;
  while (b > a && mp_lws(v[b - 1])) b--;
  if (a == b) return 1;
  uint32_t sl = a;
  while (sl < b && v[sl] != '/') sl++;
  for (uint32_t k = a; k < sl; k++)
    if (!mp_token(v[k])) return 1;
  if (sl < b) {
    if (sl + 1 == b) return 1;
    for (uint32_t k = sl + 1; k < b; k++)
      if (!mp_token(v[k])) return 1;
  }
  if (sl == a) return 1;
  *ts = a;
  *te = b;
  uint32_t i = semi;
  for (;;) {
    uint32_t ks, ke, vs, ve;
    bool q;
    const int r = mp_next_param(v, n, &i, &ks, &ke, &vs, &ve, &q);
    if (r == 1) break;
    if (r < 0) return 1;
    for (uint32_t k = ks; k < ke; k++)
      if (v[k] == '*') return 2;
    // duplicate name: compare with the parameters before this one
    uint32_t j = semi;
    for (;;) {
      uint32_t ks2, ke2, vs2, ve2;
      bool q2;
      if (mp_next_param(v, n, &j, &ks2, &ke2, &vs2, &ve2, &q2) != 0 || ks2 >= ks) break;
      if (ke2 - ks2 == ke - ks && eq_ascii_ci_both(v + ks2, v + ks, ke - ks)) return 1;
    }
    Str* out = nullptr;
    uint32_t wn0 = 0, wn1 = 0;
    while (w0[wn0]) wn0++;
    if (w1)
      while (w1[wn1]) wn1++;
    if (ke - ks == wn0 && eq_ascii_ci(v + ks, ke - ks, (const uint8_t*)w0, wn0)) out = o0;
    else if (w1 && ke - ks == wn1 && eq_ascii_ci(v + ks, ke - ks, (const uint8_t*)w1, wn1)) out = o1;
    if (out) {
      bool esc = false;
      for (uint32_t k = vs; q && k < ve; k++)
        if (v[k] == '\\' && k + 1 < ve && mp_tspecial(v[k + 1])) esc = true;
      if (!esc) {
        *out = {v + vs, ve - vs};
      } else {
        uint8_t* d = tx_alloc(t, ve - vs);
        if (!d) return 1;
        uint32_t o = 0;
        for (uint32_t k = vs; k < ve; k++) {
          if (v[k] == '\\' && k + 1 < ve && mp_tspecial(v[k + 1])) k++;
          d[o++] = v[k];
        }
        t.nb -= (ve - vs) - o;
        *out = {d, o};
      }
    }
  }
  return 0;
}

// line [*ls, *le) at s[i] without its "\r\n" / "\n"; *nx = the next line
GI_HD inline bool mp_line(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* ls, uint32_t* le, uint32_t* nx) {
  if (i >= n) return false;
  uint32_t j = i;
  while (j < n && s[j] != '\n') j++;
  *ls = i;
  *nx = j < n ? j + 1 : n;
  if (j < n && j > i && s[j - 1] == '\r') j--;
  *le = j;
  return true;
}

// textproto.CanonicalMIMEHeaderKey with its validity check
GI_HD inline bool mp_canonical(const uint8_t* k, uint32_t kn, bool* already) {
  if (kn == 0) return false;
  bool up = true, same = true;
  for (uint32_t i = 0; i < kn; i++) {
    const uint8_t c = k[i];
    if (!mp_token(c)) return false;
    const uint8_t x = (up && c >= 'a' && c <= 'z') ? c - 32 : (!up && c >= 'A' && c <= 'Z') ? c + 32 : c;
    same &= x == c;
    up = x == '-';
  }
  *already = same;
  return true;
}

GI_HD inline bool mp_is_final(const uint8_t* s, uint32_t ls, uint32_t le_nl, const uint8_t* bd, uint32_t bn,
                                   bool lf) {
  // line s[ls, le_nl) including its NL: ^--boundary--[ \t]*(NL)?$
  const uint32_t n = le_nl - ls;
  if (n < bn + 4 || s[ls] != '-' || s[ls + 1] != '-' || !bytes_equal(s + ls + 2, bd, bn) || s[ls + 2 + bn] != '-' ||
      s[ls + 3 + bn] != '-')
    return false;
  uint32_t r = ls + 4 + bn;
  while (r < le_nl && mp_lws(s[r])) r++;
  const uint32_t rest = le_nl - r;
  return rest == 0 || (lf ? (rest == 1 && s[r] == '\n') : (rest == 2 && s[r] == '\r' && s[r + 1] == '\n'));
}

// matchAfterPrefix == +1 at s[k]
GI_HD inline bool mp_after_ok(const uint8_t* s, uint32_t n, uint32_t k) {
  if (k >= n) return true;
  const uint8_t c = s[k];
  if (c == ' ' || c == '\t' || c == '\r' || c == '\n') return true;
  return c == '-' && k + 1 < n && s[k + 1] == '-';
}

// Returns an MpErr (the body-error class) or MP_OK; GI_REQ_UNSUPPORTED_BODY
// in t.flags for input outside the engine (quoted-printable parts, RFC 2231
// parameters).  *combined / *combined_set: FILES_COMBINED_SIZE.
// cand (optional, k_mpparse): every position k of a '\n' followed by
// "--" + boundary, ascending -- the delimiter search of a part's data then
// walks this list instead of every byte of the part.
// Segments (k_mpparse's part-parallel parse, block_multipart): i0 = where
// the parse starts (a delimiter line; 0 = the body), stop = a delimiter line
// at or after this position ends it with MP_SEG before that part (seg[0] =
// parts parsed, seg[1] = where that line starts).
#define MP_SEG 0xFE
template <class C>
GI_HD __noinline__ uint8_t parse_multipart(C& t, const uint8_t* s, uint32_t n, const uint8_t* ct, uint32_t ctn,
                                                uint64_t* combined, bool* combined_set,
                                                const uint32_t* cand = nullptr, uint32_t ncand = 0,
                                                uint32_t i0 = 0, uint32_t stop = 0xFFFFFFFFu, uint32_t* seg = nullptr) {
  uint32_t ci = 0;  // next candidate
  const uint32_t f_begin = t.nf;  // (FILES_SIZES entries exist only from here on)
  *combined = 0;
  *combined_set = false;
  uint32_t ts, te;
  Str bstr;
  const int mr = mp_media(t, ct, ctn, &ts, &te, "boundary", &bstr, nullptr, nullptr);
  if (mr == 2) {
    t.flags |= GI_REQ_UNSUPPORTED_BODY;
    return MP_OK;
  }
  if (mr != 0) return MP_E_MEDIA;
  if (te - ts < 10 || !eq_ascii_ci(ct + ts, 10, (const uint8_t*)"multipart/", 10)) return MP_E_NOTMP;
  if (bstr.n == 0) return MP_E_EMPTYB;
  const uint8_t* bd = bstr.p;
  const uint32_t bn = bstr.n;
  bool lf = false;
  uint32_t parts = 0, i = i0;
  uint64_t total = 0;
  if (seg) seg[0] = 0;
  for (;;) {
    // Reader.nextPart: lines until a delimiter line
    bool expect_new = false;
    for (;;) {
      uint32_t j = i;
      while (j < n && s[j] != '\n' && j - i < 4095) j++;  // bufio.Reader of 4096 bytes: ReadSlice('\n')
      if (j >= n || s[j] != '\n') {
        if (j >= n) {
          if (mp_is_final(s, i, n, bd, bn, lf)) return MP_OK;
          return MP_E_EOF;
        }
        return MP_E_BUFFULL;
      }
      const uint32_t ls = i, le = j + 1;  // the line with its '\n'
      i = j + 1;
      if (le - ls >= 2 + bn && s[ls] == '-' && s[ls + 1] == '-' && bytes_equal(s + ls + 2, bd, bn)) {
        uint32_t r = ls + 2 + bn;
        while (r < le && mp_lws(s[r])) r++;
        if (parts == 0 && le - r == 1) lf = true;  // first delimiter line ends in a bare LF: LF mode
        if (lf ? (le - r == 1) : (le - r == 2 && s[r] == '\r')) {
          if (ls >= stop) {
            seg[1] = ls;
            return MP_SEG;
          }
          break;
        }
      }
      if (mp_is_final(s, ls, le, bd, bn, lf)) return MP_OK;
      if (expect_new) return MP_E_EXPECT;
      if (parts == 0) continue;
      if (lf ? (le - ls == 1) : (le - ls == 2 && s[ls] == '\r')) {
        expect_new = true;
        continue;
      }
      return MP_E_UNEXP;
    }
    parts++;
    if (seg) seg[0] = parts;
    // textproto.ReadMIMEHeader: FK_PART_HEADER fields (key, value) for now
    const uint32_t h0 = t.nf;
    uint8_t herr = MP_OK;
    for (bool first = true; herr == MP_OK; first = false) {
      uint32_t ls, le, nx;
      if (!mp_line(s, n, i, &ls, &le, &nx) || (first && le > ls && mp_lws(s[ls]))) {
        herr = MP_E_HDR;
        break;
      }
      i = nx;
      if (le == ls) break;
      uint32_t a = ls, b = le;
      while (a < b && mp_lws(s[a])) a++;
      while (b > a && mp_lws(s[b - 1])) b--;
      const uint8_t* kv = s + a;
      uint32_t kvn = b - a;
      if (i < n && mp_lws(s[i])) {  // continuation lines: joined with one space
        uint32_t cap = kvn, p = i;
        for (;;) {
          uint32_t l2, e2, x2;
          if (!(p < n && mp_lws(s[p])) || !mp_line(s, n, p, &l2, &e2, &x2)) break;
          cap += 1 + (e2 - l2);
          p = x2;
        }
        uint8_t* d = tx_alloc(t, cap);
        if (!d) return MP_OK;  // arena overflow (flagged)
        for (uint32_t k = 0; k < kvn; k++) d[k] = kv[k];
        uint32_t o = kvn;
        while (i < n && mp_lws(s[i])) {
          uint32_t l2, e2, x2;
          mp_line(s, n, i, &l2, &e2, &x2);
          i = x2;
          while (l2 < e2 && mp_lws(s[l2])) l2++;
          while (e2 > l2 && mp_lws(s[e2 - 1])) e2--;
          d[o++] = ' ';
          for (uint32_t k = l2; k < e2; k++) d[o++] = s[k];
        }
        t.nb -= cap - o;
        kv = d;
        kvn = o;
      }
      uint32_t c = 0;
      while (c < kvn && kv[c] != ':') c++;
      bool canon = false;
      if (c == kvn || !mp_canonical(kv, c, &canon)) herr = MP_E_HDR;
      for (uint32_t k = c + 1; k < kvn && herr == MP_OK; k++) {
        const uint8_t x = kv[k];
        if (!(x >= 0x20 || x == '\t') || x == 0x7F) herr = MP_E_HDR;
      }
      if (herr) break;
      const uint8_t* key = kv;
      if (!canon) {
        uint8_t* d = tx_alloc(t, c);
        if (!d) return MP_OK;
        bool up = true;
        for (uint32_t k = 0; k < c; k++) {
          const uint8_t x = kv[k];
          d[k] = (up && x >= 'a' && x <= 'z') ? x - 32 : (!up && x >= 'A' && x <= 'Z') ? x + 32 : x;
          up = d[k] == '-';
        }
        key = d;
      }
      uint32_t vs = c + 1;
      while (vs < kvn && mp_lws(kv[vs])) vs++;
      add_field(t, FK_PART_HEADER, key, c, kv + vs, kvn - vs);
    }
    if (herr) {  // NextPart's error: this part added nothing
      t.nf = h0;
      return herr;
    }
    if (t.flags & GI_REQ_ERROR_MASK) return MP_OK;
    const uint32_t h1 = t.nf;
    // first Content-Disposition / Content-Transfer-Encoding
    Str cd{CS_ZERO, 0};
    bool have_cd = false;
    for (uint32_t f = h0; f < h1; f++) {
      const Field& F = t.fields[f];
      if (!have_cd && F.kn == 19 && bytes_equal(F.k, (const uint8_t*)"Content-Disposition", 19)) {
        cd = {F.v, F.vn};
        have_cd = true;
      }
      if (F.kn == 25 && bytes_equal(F.k, (const uint8_t*)"Content-Transfer-Encoding", 25)) {
        if (F.vn == 16 && eq_ascii_ci(F.v, 16, (const uint8_t*)"quoted-printable", 16)) {
          t.flags |= GI_REQ_UNSUPPORTED_BODY;
          return MP_OK;
        }
        break;  // Header.Get: the first value decides
      }
    }
    // the part's data: up to the first NL + "--" + boundary + terminator
    uint32_t end = 0xFFFFFFFFu;
    if (n - i >= 2 + bn && s[i] == '-' && s[i + 1] == '-' && bytes_equal(s + i + 2, bd, bn) &&
        mp_after_ok(s, n, i + 2 + bn)) {
      end = i;
    } else if (cand) {  // the same first match, from the candidate list
      while (ci < ncand && cand[ci] < i + (lf ? 0u : 1u)) ci++;
      for (uint32_t c = ci; c < ncand; c++) {
        const uint32_t k = cand[c];  // '\n'; the delimiter starts at k (LF) or k - 1 (CRLF)
        if (!lf && s[k - 1] != '\r') continue;
        if (mp_after_ok(s, n, k + 3 + bn)) {
          end = lf ? k : k - 1;
          ci = c;
          break;
        }
      }
    } else {
      const uint32_t pl = (lf ? 1u : 2u) + 2 + bn;
      for (uint32_t k = i; k + pl <= n; k++) {
        if (s[k] != (lf ? '\n' : '\r')) continue;
        if (!lf && s[k + 1] != '\n') continue;
        const uint32_t d0 = k + (lf ? 1 : 2);
        if (s[d0] == '-' && s[d0 + 1] == '-' && bytes_equal(s + d0 + 2, bd, bn) && mp_after_ok(s, n, d0 + 2 + bn)) {
          end = k;
          break;
        }
      }
    }
    if (end == 0xFFFFFFFFu) {  // the part's reader hits EOF: io.ReadAll / io.Copy fails before any Add
      t.nf = h0;
      return MP_E_DATA;
    }
    const uint8_t* data = s + i;
    const uint32_t dn = end - i;
    i = end;
    // disposition: FormName (form-data only) and the filename parameter
    Str name{CS_ZERO, 0}, fname{CS_ZERO, 0};
    if (have_cd) {
      uint32_t dts, dte;
      Str nm, fn;
      const int dr = mp_media(t, cd.p, cd.n, &dts, &dte, "name", &nm, "filename", &fn);
      if (dr == 2) {
        t.flags |= GI_REQ_UNSUPPORTED_BODY;
        return MP_OK;
      }
      if (dr == 0) {
        fname = fn;
        if (dte - dts == 9 && eq_ascii_ci(cd.p + dts, 9, (const uint8_t*)"form-data", 9)) name = nm;
      }
    }
    // MULTIPART_PART_HEADERS: (name, "Key: value"), keys sorted (stable)
    for (uint32_t f = h0; f < h1; f++) {
      Field& F = t.fields[f];
      uint8_t* d = tx_alloc(t, F.kn + 2 + F.vn);
      if (!d) return MP_OK;
      for (uint32_t k = 0; k < F.kn; k++) d[k] = F.k[k];
      d[F.kn] = ':';
      d[F.kn + 1] = ' ';
      for (uint32_t k = 0; k < F.vn; k++) d[F.kn + 2 + k] = F.v[k];
      F.v = d;
      F.vn = F.kn + 2 + F.vn;  // F.k still the key: the sort below reads it
    }
    for (uint32_t f = h0 + 1; f < h1; f++) {
      const Field x = t.fields[f];
      uint32_t g = f;
      while (g > h0) {
        const Field& y = t.fields[g - 1];
        // y.k > x.k (bytewise)?
        const uint32_t m = min(y.kn, x.kn);
        int cmp = 0;
        for (uint32_t k = 0; k < m && !cmp; k++) cmp = (int)y.k[k] - (int)x.k[k];
        if (!cmp) cmp = (int)y.kn - (int)x.kn;
        if (cmp <= 0) break;
        t.fields[g] = y;
        g--;
      }
      t.fields[g] = x;
    }
    for (uint32_t f = h0; f < h1; f++) {
      t.fields[f].k = name.p;
      t.fields[f].kn = name.n;
    }
    total += dn;
    if (fname.n) {
      add_field(t, FK_FILE, CS_ZERO, 0, fname.p, fname.n);
      uint8_t* sz = tx_alloc(t, 24);
      if (!sz) return MP_OK;
      const uint32_t szn = go_itoa((int64_t)dn, sz);
      t.nb -= 24 - szn;
      bool set = false;
      for (uint32_t f = f_begin; f < t.nf && !set; f++) {  // FILES_SIZES.SetIndex(file name, 0, size)
        Field& F = t.fields[f];
        if (F.kind == FK_FILE_SIZE && F.kn == fname.n && eq_ascii_ci_both(F.k, fname.p, fname.n)) {
          F.v = sz;
          F.vn = szn;
          set = true;
        }
      }
      if (!set) add_field(t, FK_FILE_SIZE, fname.p, fname.n, sz, szn);
      add_field(t, FK_FILE_NAME, CS_ZERO, 0, name.p, name.n);
    } else {
      add_field(t, FK_ARG_POST, name.p, name.n, data, dn);
    }
    if (t.flags & GI_REQ_ERROR_MASK) return MP_OK;
    *combined = total;
    *combined_set = true;
  }
}

// ------------------------------------------------------------ XML body
// [upstream coraza internal/bodyprocessors/xml.go readXML over Go's
// encoding/xml Decoder, Strict = false, AutoClose = HTMLAutoClose, Entity =
// HTMLEntity]; oracle/xmlbody.py states the same paths.  Output fields
// (FK_XML): key "//@*" for every attribute value of every start element,
// then key "/*" for every strings.TrimSpace'd non-empty character-data token,
// each in document order.  A decoder error -> no fields, *msg = "XML: " +
// err.Error() in the arena, return 1.  Non-ASCII XML names (Go's XML name
// range tables) -> GI_REQ_UNSUPPORTED_BODY.  ws: cap words of scratch for the
// element stack and the text list.
struct XName {
  uint32_t so, sn, lo, ln;  // prefix [so, so + sn) and local part [lo, lo + ln) in the body
};

GI_HD inline bool xml_name_byte(uint8_t c) {
  return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '_' || c == ':' ||
         c == '.' || c == '-';
}
GI_HD inline bool xml_in_range(uint32_t r) {
  return r == 0x09 || r == 0x0A || r == 0x0D || (r >= 0x20 && r <= 0xD7FF) || (r >= 0xE000 && r <= 0xFFFD) ||
         (r >= 0x10000 && r <= 0x10FFFF);
}
GI_HD inline bool go_is_space(uint32_t r) {  // unicode.IsSpace
  return r == 0x09 || r == 0x0A || r == 0x0B || r == 0x0C || r == 0x0D || r == 0x20 || r == 0x85 || r == 0xA0 ||
         r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 || r == 0x202F || r == 0x205F ||
         r == 0x3000;
}
// HTML 4.01 entity by name (sorted table): code point or -1
GI_HD int32_t html_entity(const uint8_t* nm, uint32_t n) {
  uint32_t lo = 0, hi = GI_N_HTML_ENT;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint8_t* e = (const uint8_t*)kHtmlEntPool + kHtmlEnt[mid][0];
    const uint32_t en = kHtmlEnt[mid][1];
    int c = 0;
    for (uint32_t k = 0; k < en && k < n && !c; k++) c = (int)e[k] - (int)nm[k];
    if (!c) c = (int)en - (int)n;
    if (c == 0) return (int32_t)kHtmlEnt[mid][2];
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return -1;
}

template <class C>
struct XmlDec {
  C& t;
  const uint8_t* s;
  uint32_t n, i, line;
  int err;          // 0 none, 1 decoder error (msg set), 2 unsupported, 3 arena overflow
  uint32_t mo, ml;  // error message in the arena
  GI_HD XmlDec(C& tt, const uint8_t* ss, uint32_t nn) : t(tt), s(ss), n(nn), i(0), line(1), err(0), mo(0), ml(0) {}
  GI_HD int getc() {
    if (i >= n) return -1;
    const uint8_t b = s[i++];
    if (b == '\n') line++;
    return b;
  }
  GI_HD void ungetc(int b) {
    if (b == '\n') line--;
    i--;
  }
  // message pieces
  GI_HD void put(const char* p) {
    for (; *p && err != 3; p++) putb((uint8_t)*p);
  }
  GI_HD void putb(uint8_t b) {
    if (t.nb + 1 > t.cap_b) {
      err = 3;
      return;
    }
    t.bytes[t.nb++] = b;
    ml++;
  }
  GI_HD void putn(const uint8_t* p, uint32_t k) {
    for (uint32_t q = 0; q < k; q++) putb(p[q]);
  }
  GI_HD void putu(uint32_t v) {
    uint8_t b[12];
    const uint32_t k = go_itoa((int64_t)v, b);
    putn(b, k);
  }
  GI_HD void begin_msg(bool syntax) {
    err = 1;
    mo = t.nb;
    ml = 0;
    put("XML: ");
    if (syntax) {
      put("XML syntax error on line ");
      putu(line);
      put(": ");
    }
  }
  GI_HD void syntax(const char* m) {
    begin_msg(true);
    put(m);
  }
  GI_HD int mustgetc() {
    const int b = getc();
    if (b < 0) syntax("unexpected EOF");
    return b;
  }
  GI_HD void space() {
    for (;;) {
      const int b = getc();
      if (b < 0) return;
      if (b != ' ' && b != '\r' && b != '\n' && b != '\t') {
        ungetc(b);
        return;
      }
    }
  }
  // readName over the body: [*a, *e); false (nothing read) or err
  GI_HD bool read_name(uint32_t* a, uint32_t* e) {
    int b = mustgetc();
    if (b < 0) return false;
    if (b < 0x80 && !xml_name_byte((uint8_t)b)) {
      ungetc(b);
      return false;
    }
    *a = i - 1;
    for (;;) {
      b = mustgetc();
      if (b < 0) return false;
      if (b < 0x80 && !xml_name_byte((uint8_t)b)) {
        ungetc(b);
        break;
      }
    }
    *e = i;
    return true;
  }
  // isName for a name read by read_name (err 2 when it has non-ASCII bytes)
  GI_HD bool is_name(uint32_t a, uint32_t e) {
    if (e == a) return false;
    for (uint32_t k = a; k < e; k++)
      if (s[k] >= 0x80) {
        err = 2;
        return false;
      }
    const uint8_t c = s[a];
    return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_' || c == ':';
  }
  // name(): false without a name (err unset) or on error
  GI_HD bool name(uint32_t* a, uint32_t* e) {
    if (!read_name(a, e)) return false;
    if (!is_name(*a, *e)) {
      if (err == 2) return false;
      begin_msg(true);
      put("invalid XML name: ");
      putn(s + *a, *e - *a);
      return false;
    }
    return true;
  }
  GI_HD bool nsname(XName* x) {
    uint32_t a, e;
    if (!name(&a, &e)) return false;
    uint32_t colons = 0, c = e;
    for (uint32_t k = a; k < e; k++)
      if (s[k] == ':') {
        if (!colons) c = k;
        colons++;
      }
    if (colons > 1) return false;
    if (!colons || c == a || c + 1 == e) {
      *x = {a, 0, a, e - a};
    } else {
      *x = {a, c - a, c + 1, e - c - 1};
    }
    return true;
  }
  // text(quote, cdata): the decoded bytes appended to the arena at *o (length
  // *len); false on error.  Decoded text is never longer than its input.
  GI_HD bool text(int quote, bool cdata, uint32_t* o, uint32_t* len) {
    uint8_t b0 = 0, b1 = 0;
    uint32_t trunc = 0;
    const uint32_t start = t.nb;
    auto wr = [&](uint8_t c) {
      if (t.nb + 1 > t.cap_b) {
        err = 3;
        return false;
      }
      t.bytes[t.nb++] = c;
      return true;
    };
    for (;;) {
      int b = getc();
      if (b < 0) {
        if (cdata) {
          syntax("unexpected EOF in CDATA section");
          return false;
        }
        break;
      }
      if (quote < 0 && b0 == ']' && b1 == ']' && b == '>') {
        if (cdata) {
          trunc = 2;
          break;
        }
        syntax("unescaped ]]> not in CDATA section");
        return false;
      }
      if (b == '<' && !cdata) {
        if (quote >= 0) {
          syntax("unescaped < inside quoted string");
          return false;
        }
        ungetc(b);
        break;
      }
      if (quote >= 0 && b == quote) break;
      if (b == '&' && !cdata) {
        const uint32_t before = t.nb;
        if (!wr('&')) return false;
        int32_t cp = -1;
        b = mustgetc();
        if (b < 0) return false;
        if (b == '#') {
          if (!wr('#')) return false;
          b = mustgetc();
          if (b < 0) return false;
          uint32_t base = 10;
          if (b == 'x') {
            base = 16;
            if (!wr('x')) return false;
            b = mustgetc();
            if (b < 0) return false;
          }
          const uint32_t dstart = t.nb;
          uint64_t v = 0;
          bool big = false;
          while ((b >= '0' && b <= '9') || (base == 16 && ((b >= 'a' && b <= 'f') || (b >= 'A' && b <= 'F')))) {
            if (!wr((uint8_t)b)) return false;
            const uint32_t dv = b <= '9' ? b - '0' : ((b | 0x20) - 'a' + 10);
            if (v > 0x10FFFFull) big = true;
            else v = v * base + dv;
            b = mustgetc();
            if (b < 0) return false;
          }
          if (b != ';') {
            ungetc(b);
          } else {
            if (!wr(';')) return false;
            if (t.nb - 1 > dstart && !big && v <= 0x10FFFF) cp = (v >= 0xD800 && v <= 0xDFFF) ? 0xFFFD : (int32_t)v;
          }
        } else {
          ungetc(b);
          uint32_t a, e;
          const bool got = read_name(&a, &e);
          if (err) return false;
          if (got)
            for (uint32_t k = a; k < e; k++)
              if (!wr(s[k])) return false;
          b = mustgetc();
          if (b < 0) return false;
          if (b != ';') {
            ungetc(b);
          } else {
            const uint8_t* nm = t.bytes + before + 1;
            const uint32_t nn = t.nb - before - 1;
            if (!wr(';')) return false;
            bool ascii = nn > 0;
            for (uint32_t k = 0; k < nn; k++) ascii &= nm[k] < 0x80;
            const uint8_t c0 = nn ? nm[0] : 0;
            if (ascii && ((c0 >= 'A' && c0 <= 'Z') || (c0 >= 'a' && c0 <= 'z') || c0 == '_' || c0 == ':')) {
              if (nn == 2 && nm[0] == 'l' && nm[1] == 't') cp = '<';
              else if (nn == 2 && nm[0] == 'g' && nm[1] == 't') cp = '>';
              else if (nn == 3 && nm[0] == 'a' && nm[1] == 'm' && nm[2] == 'p') cp = '&';
              else if (nn == 4 && nm[0] == 'a' && nm[1] == 'p' && nm[2] == 'o' && nm[3] == 's') cp = '\'';
              else if (nn == 4 && nm[0] == 'q' && nm[1] == 'u' && nm[2] == 'o' && nm[3] == 't') cp = '"';
              else cp = html_entity(nm, nn);
            }
          }
        }
        if (cp >= 0) {  // replace "&...;" by the rune
          t.nb = before;
          uint8_t enc[4];
          const uint32_t k = encode_rune((uint32_t)cp, enc);
          for (uint32_t q = 0; q < k; q++)
            if (!wr(enc[q])) return false;
        }
        b0 = b1 = 0;
        continue;  // non-strict: an unknown entity stays as written
      }
      if (b == '\r') {
        if (!wr('\n')) return false;
      } else if (!(b1 == '\r' && b == '\n')) {
        if (!wr((uint8_t)b)) return false;
      }
      b0 = b1;
      b1 = (uint8_t)b;
    }
    const uint32_t dn = t.nb - start - trunc;
    t.nb -= trunc;
    for (uint32_t k = 0; k < dn;) {  // disallowed characters
      uint32_t w;
      const uint32_t r = decode_rune(t.bytes + start, dn, k, &w);
      if (r == 0xFFFD && w == 1) {
        syntax("invalid UTF-8");
        return false;
      }
      k += w;
      if (!xml_in_range(r)) {
        begin_msg(true);
        put("illegal character code U+");
        uint8_t hx[8];
        uint32_t hn = 0;
        for (int sh = 20; sh >= 0; sh -= 4) {
          const uint32_t d = (r >> sh) & 15;
          if (hn || d || sh < 16) hx[hn++] = (uint8_t)(d < 10 ? '0' + d : 'A' + d - 10);
        }
        putn(hx, hn);
        return false;
      }
    }
    *o = start;
    *len = dn;
    return true;
  }
  GI_HD bool attrval(uint32_t* o, uint32_t* len) {
    int b = mustgetc();
    if (b < 0) return false;
    if (b == '"' || b == '\'') return text(b, false, o, len);
    ungetc(b);
    const uint32_t a = i;
    for (;;) {
      b = mustgetc();
      if (b < 0) return false;
      if ((b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z') || (b >= '0' && b <= '9') || b == '_' || b == ':' ||
          b == '-')
        continue;
      ungetc(b);
      break;
    }
    *o = 0xFFFFFFFFu;  // the value is s[a, i): in the body, not the arena
    *len = i - a;
    return true;
  }
};

enum XTok : uint8_t { XT_NONE = 0, XT_START, XT_END, XT_CHARS, XT_OTHER };

// encoding/xml procInst(param, s): the quoted value of param="..." in s
GI_HD bool xml_proc_inst(const uint8_t* s, uint32_t n, const char* param, uint32_t* vo, uint32_t* vn) {
  uint32_t lp = 0;
  while (param[lp]) lp++;  // includes the '='
  uint32_t i = 0;
  uint8_t sep = 0;
  while (i < n) {
    int64_t k = -1;
    for (uint32_t q = i; q + lp <= n && k < 0; q++) {
      bool eq = true;
      for (uint32_t z = 0; z < lp && eq; z++) eq = s[q + z] == (uint8_t)param[z];
      if (eq) k = q - i;
    }
    if (k < 0 || lp + (uint32_t)k >= n - i) return false;
    const uint8_t c = s[i + lp + k];
    i += lp + (uint32_t)k + 1;
    if (c == '\'' || c == '"') {
      sep = c;
      break;
    }
  }
  if (!sep) return false;
  for (uint32_t j = i; j < n; j++)
    if (s[j] == sep) {
      *vo = i;
      *vn = j - i;
      return true;
    }
  return false;
}

GI_HD inline bool xml_autoclose(const uint8_t* s, uint32_t lo, uint32_t ln) {
  const char* names[13] = {"basefont", "br", "area", "link", "img", "param", "hr", "input", "col", "frame",
                           "isindex", "base", "meta"};
  for (int k = 0; k < 13; k++) {
    uint32_t m = 0;
    while (names[k][m]) m++;
    if (m == ln && eq_ascii_ci(s + lo, ln, (const uint8_t*)names[k], m)) return true;
  }
  return false;
}

template <class C>
GI_HD __noinline__ int parse_xml(C& t, const uint8_t* s, uint32_t n, uint32_t* ws, uint32_t ws_words, Str* msg) {
  XmlDec<C> d(t, s, n);
  const uint32_t nf0 = t.nf, nb0 = t.nb;
  // ws: element stack (XName, 4 words each) from the front, text list ((off, len) pairs) from the back
  XName* stk = (XName*)ws;
  uint32_t depth = 0, ntext = 0;
  const uint32_t cap_items = ws_words / 4;  // stack entries + text pairs / 2 share the space
  uint32_t* texts = ws + ws_words;          // grows down: texts[-2(k+1)], texts[-2(k+1)+1]
  bool need_close = false, have_next = false;
  XName to_close{}, next_name{};
  uint8_t next_kind = XT_NONE;
  auto fail_ret = [&]() -> int {
    t.nf = nf0;
    if (d.err == 1) {
      *msg = {t.bytes + d.mo, d.ml};
      return 1;
    }
    t.nb = nb0;
    t.flags |= d.err == 2 ? GI_REQ_UNSUPPORTED_BODY : GI_REQ_OVERFLOW;
    return 2;
  };
  for (;;) {
    uint8_t kind = XT_NONE;
    XName nm{};
    if (have_next) {
      kind = next_kind;
      nm = next_name;
      have_next = false;
    } else {
      // ---- rawToken
      if (need_close) {
        need_close = false;
        kind = XT_END;
        nm = to_close;
      } else {
        int b = d.getc();
        if (b < 0) {  // EOF
          if (depth) {
            d.syntax("unexpected EOF");
            return fail_ret();
          }
          break;
        }
        if (b != '<') {
          d.ungetc(b);
          uint32_t o, len;
          if (!d.text(-1, false, &o, &len)) return fail_ret();
          kind = XT_CHARS;
          nm = {o, len, 0, 0};
        } else {
          b = d.mustgetc();
          if (b < 0) return fail_ret();
          if (b == '/') {
            if (!d.nsname(&nm)) {
              if (!d.err) d.syntax("expected element name after </");
              return fail_ret();
            }
            d.space();
            b = d.mustgetc();
            if (b < 0) return fail_ret();
            if (b != '>') {
              d.begin_msg(true);
              d.put("invalid characters between </");
              d.putn(s + nm.lo, nm.ln);
              d.put(" and >");
              return fail_ret();
            }
            kind = XT_END;
          } else if (b == '?') {
            uint32_t ta, te;
            if (!d.name(&ta, &te)) {
              if (!d.err) d.syntax("expected target name after <?");
              return fail_ret();
            }
            d.space();
            const uint32_t c0 = d.i;
            uint8_t p0 = 0;
            for (;;) {
              b = d.mustgetc();
              if (b < 0) return fail_ret();
              if (p0 == '?' && b == '>') break;
              p0 = (uint8_t)b;
            }
            const uint32_t cn = d.i - 2 - c0;
            if (te - ta == 3 && s[ta] == 'x' && s[ta + 1] == 'm' && s[ta + 2] == 'l') {
              uint32_t vo, vn;
              if (xml_proc_inst(s + c0, cn, "version=", &vo, &vn) && vn &&
                  !(vn == 3 && s[c0 + vo] == '1' && s[c0 + vo + 1] == '.' && s[c0 + vo + 2] == '0')) {
                d.begin_msg(false);
                d.put("xml: unsupported version \"");
                d.putn(s + c0 + vo, vn);
                d.put("\"; only version 1.0 is supported");
                return fail_ret();
              }
              if (xml_proc_inst(s + c0, cn, "encoding=", &vo, &vn) && vn &&
                  !(vn == 5 && eq_ascii_ci(s + c0 + vo, 5, (const uint8_t*)"utf-8", 5))) {
                d.begin_msg(false);
                d.put("xml: encoding \"");
                d.putn(s + c0 + vo, vn);
                d.put("\" declared but Decoder.CharsetReader is nil");
                return fail_ret();
              }
            }
            kind = XT_OTHER;
          } else if (b == '!') {
            b = d.mustgetc();
            if (b < 0) return fail_ret();
            if (b == '-') {
              b = d.mustgetc();
              if (b < 0) return fail_ret();
              if (b != '-') {
                d.syntax("invalid sequence <!- not part of <!--");
                return fail_ret();
              }
              uint8_t q0 = 0, q1 = 0;
              for (;;) {
                b = d.mustgetc();
                if (b < 0) return fail_ret();
                if (q0 == '-' && q1 == '-') {
                  if (b != '>') {
                    d.syntax("invalid sequence \"--\" not allowed in comments");
                    return fail_ret();
                  }
                  break;
                }
                q0 = q1;
                q1 = (uint8_t)b;
              }
              kind = XT_OTHER;
            } else if (b == '[') {
              const char* cd = "CDATA[";
              for (int k = 0; k < 6; k++) {
                b = d.mustgetc();
                if (b < 0) return fail_ret();
                if (b != cd[k]) {
                  d.syntax("invalid <![ sequence");
                  return fail_ret();
                }
              }
              uint32_t o, len;
              if (!d.text(-1, true, &o, &len)) return fail_ret();
              kind = XT_CHARS;
              nm = {o, len, 0, 0};
            } else {  // a directive
              uint8_t inq = 0;
              int depth2 = 0;
              for (;;) {
                b = d.mustgetc();
                if (b < 0) return fail_ret();
                if (inq == 0 && b == '>' && depth2 == 0) break;
                for (bool again = true; again;) {  // HandleB
                  again = false;
                  if (b == inq) {
                    inq = 0;
                  } else if (inq != 0) {
                  } else if (b == '\'' || b == '"') {
                    inq = (uint8_t)b;
                  } else if (b == '>') {
                    depth2--;
                  } else if (b == '<') {
                    const char* cm = "!--";
                    for (int k = 0; k < 3; k++) {
                      b = d.mustgetc();
                      if (b < 0) return fail_ret();
                      if (b != cm[k]) {
                        depth2++;
                        again = true;
                        break;
                      }
                    }
                    if (!again) {
                      uint8_t q0 = 0, q1 = 0;
                      for (;;) {
                        b = d.mustgetc();
                        if (b < 0) return fail_ret();
                        if (q0 == '-' && q1 == '-' && b == '>') break;
                        q0 = q1;
                        q1 = (uint8_t)b;
                      }
                    }
                  }
                }
              }
              kind = XT_OTHER;
            }
          } else {  // an open element
            d.ungetc(b);
            if (!d.nsname(&nm)) {
              if (!d.err) d.syntax("expected element name after <");
              return fail_ret();
            }
            bool empty = false;
            for (;;) {
              d.space();
              b = d.mustgetc();
              if (b < 0) return fail_ret();
              if (b == '/') {
                empty = true;
                b = d.mustgetc();
                if (b < 0) return fail_ret();
                if (b != '>') {
                  d.syntax("expected /> in element");
                  return fail_ret();
                }
                break;
              }
              if (b == '>') break;
              d.ungetc(b);
              XName an;
              if (!d.nsname(&an)) {
                if (!d.err) d.syntax("expected attribute name in element");
                return fail_ret();
              }
              d.space();
              b = d.mustgetc();
              if (b < 0) return fail_ret();
              const uint8_t* vp;
              uint32_t vn;
              if (b != '=') {  // non-strict: the value is the name's local part
                d.ungetc(b);
                vp = s + an.lo;
                vn = an.ln;
              } else {
                d.space();
                uint32_t o, len;
                if (!d.attrval(&o, &len)) return fail_ret();
                vp = o == 0xFFFFFFFFu ? s + d.i - len : t.bytes + o;
                vn = len;
              }
              add_field(t, FK_XML, CS_XML_ATTRS, 4, vp, vn);
              if (t.flags & GI_REQ_ERROR_MASK) {
                d.err = 3;
                return fail_ret();
              }
            }
            if (empty) {
              need_close = true;
              to_close = nm;
            }
            kind = XT_START;
          }
        }
      }
    }
    // ---- Token(): autoClose, element stack
    if (depth && xml_autoclose(s, stk[depth - 1].lo, stk[depth - 1].ln)) {
      const XName& top = stk[depth - 1];
      if (!(kind == XT_END && nm.ln == top.ln && eq_ascii_ci_both(s + nm.lo, s + top.lo, top.ln))) {
        have_next = true;
        next_kind = kind;
        next_name = nm;
        kind = XT_END;
        nm = top;
      }
    }
    if (kind == XT_START) {
      if (depth >= cap_items || 4ull * (depth + 1) + 2ull * ntext > ws_words) {
        d.err = 3;
        return fail_ret();
      }
      stk[depth++] = nm;
    } else if (kind == XT_END) {
      if (!depth) {
        d.begin_msg(true);
        d.put("unexpected end element </");
        d.putn(s + nm.lo, nm.ln);
        d.put(">");
        return fail_ret();
      }
      const XName top = stk[--depth];
      if (!(top.ln == nm.ln && bytes_equal(s + top.lo, s + nm.lo, nm.ln))) {
        need_close = true;
        to_close = nm;
      } else if (!(top.sn == nm.sn && bytes_equal(s + top.so, s + nm.so, nm.sn))) {
        d.begin_msg(true);
        d.put("element <");
        d.putn(s + top.lo, top.ln);
        d.put("> in space ");
        d.putn(s + top.so, top.sn);
        d.put(" closed by </");
        d.putn(s + nm.lo, nm.ln);
        d.put("> in space ");
        if (nm.sn) d.putn(s + nm.so, nm.sn);
        else d.put("\"\"");
        return fail_ret();
      }
    } else if (kind == XT_CHARS) {  // strings.TrimSpace; keep a non-empty text for the "/*" list
      const uint8_t* p = t.bytes + nm.so;
      uint32_t a = 0, e = nm.sn;
      while (a < e) {
        uint32_t w;
        const uint32_t r = decode_rune(p, e, a, &w);
        if ((r == 0xFFFD && w == 1) || !go_is_space(r)) break;
        a += w;
      }
      while (e > a) {
        uint32_t k = e - 1;
        while (k > a && e - k < 4 && (p[k] & 0xC0) == 0x80) k--;
        uint32_t w;
        uint32_t r = decode_rune(p, e, k, &w);
        if (k + w != e) {
          k = e - 1;
          r = 0xFFFD;
          w = 1;
        }
        if ((r == 0xFFFD && w == 1) || !go_is_space(r)) break;
        e = k;
      }
      if (e > a) {
        if (4ull * depth + 2ull * (ntext + 1) > ws_words) {
          d.err = 3;
          return fail_ret();
        }
        ntext++;
        texts[-2 * (int64_t)ntext] = nm.so + a;
        texts[-2 * (int64_t)ntext + 1] = e - a;
      }
    }
  }
  for (uint32_t k = 1; k <= ntext; k++) {
    add_field(t, FK_XML, CS_XML_TEXT, 2, t.bytes + texts[-2 * (int64_t)k], texts[-2 * (int64_t)k + 1]);
    if (t.flags & GI_REQ_ERROR_MASK) {
      d.err = 3;
      return fail_ret();
    }
  }
  return 0;
}

// net/url shouldEscape(c, encodePath)
GI_HD inline bool should_escape_path(uint8_t c) {
  if (isalnum_(c)) return false;
  switch (c) {
    case '-': case '_': case '.': case '~': return false;
    case '$': case '&': case '+': case ',': case '/': case ':': case ';': case '=': case '?': case '@':
      return c == '?';
  }
  return true;
}
GI_HD inline bool valid_encoded_path_char(uint8_t c) {
  switch (c) {
    case '!': case '$': case '&': case '\'': case '(': case ')': case '*': case '+': case ',': case ';':
    case '=': case ':': case '@': case '[': case ']': case '%':
      return true;
  }
  return !should_escape_path(c);
}

// ProcessURI [upstream corazawaf/transaction.go] + Go net/url Parse/String
// Go net/url shouldEscape for the host and userinfo modes (path: should_escape_path)
GI_HD inline bool should_escape_host(uint8_t c) {
  if (isalnum_(c)) return false;
  switch (c) {
    case '!': case '$': case '&': case '\'': case '(': case ')': case '*': case '+': case ',': case ';':
    case '=': case ':': case '[': case ']': case '<': case '>': case '"':
    case '-': case '_': case '.': case '~':
      return false;
  }
  return true;
}
GI_HD inline bool should_escape_user(uint8_t c) {
  if (isalnum_(c)) return false;
  switch (c) {
    case '-': case '_': case '.': case '~': return false;
    case '$': case '&': case '+': case ',': case ';': case '=': return false;
    case '/': case ':': case '?': case '@': return true;
  }
  return true;
}
// net/url unescape's validation pass: mode 0 path / userinfo, 1 host (%XX only
// for non-ASCII bytes or %25; no ASCII byte the host mode escapes)
GI_HD inline bool url_unescape_ok(const uint8_t* s, uint32_t n, int mode) {
  for (uint32_t i = 0; i < n;) {
    if (s[i] == '%') {
      if (i + 2 >= n || !ishex(s[i + 1]) || !ishex(s[i + 2])) return false;
      if (mode == 1 && hexv(s[i + 1]) < 8 && !(s[i + 1] == '2' && s[i + 2] == '5')) return false;
      i += 3;
    } else {
      if (mode == 1 && s[i] < 0x80 && should_escape_host(s[i])) return false;
      i++;
    }
  }
  return true;
}
GI_HD inline uint32_t url_unescape(const uint8_t* s, uint32_t n, uint8_t* d) {
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (s[i] == '%') {
      d[o++] = x2c(s[i + 1], s[i + 2]);
      i += 2;
    } else {
      d[o++] = s[i];
    }
  }
  return o;
}
// escape(s, mode) appended at d (mode 0 path, 1 host, 2 userinfo); returns the length
GI_HD inline uint32_t url_escape(const uint8_t* s, uint32_t n, int mode, uint8_t* d) {
  const char* hx = "0123456789ABCDEF";
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    const bool e = mode == 0 ? should_escape_path(c) : mode == 1 ? should_escape_host(c) : should_escape_user(c);
    if (e) {
      d[o++] = '%';
      d[o++] = hx[c >> 4];
      d[o++] = hx[c & 15];
    } else {
      d[o++] = c;
    }
  }
  return o;
}
GI_HD inline bool valid_port(const uint8_t* s, uint32_t n) {  // "" or ":" digits
  if (n == 0) return true;
  if (s[0] != ':') return false;
  for (uint32_t i = 1; i < n; i++)
    if (s[i] < '0' || s[i] > '9') return false;
  return true;
}

// [upstream corazawaf/transaction.go ProcessURI + Go net/url Parse / String]:
// REQUEST_URI_RAW; the '#'-stripped target through url.Parse: REQUEST_URI =
// URL.String(), REQUEST_FILENAME = URL.Path, QUERY_STRING = URL.RawQuery,
// ARGS_GET; a Parse error leaves REQUEST_URI / REQUEST_FILENAME = the target
// and no GET args.  Every form Parse accepts: origin, absolute
// ("http://user@h:80/p"), scheme-relative ("//h/p"), asterisk, opaque
// ("mailto:x"), relative ("a/b").  An IPv6 zone ("[fe80::1%25en0]") sets
// GI_REQ_UNSUPPORTED_URI (the oracle flags it the same way).
GI_HD bool process_uri(Tx& t, const uint8_t* uri, uint32_t un) {
  t.single[S_REQUEST_URI_RAW] = {uri, un};
  uint32_t n = un;
  for (uint32_t i = 0; i < un; i++)
    if (uri[i] == '#') { n = i; break; }
  Str path{uri, n}, query{uri, 0};
  bool err = false;
  for (uint32_t i = 0; i < n; i++)
    if (uri[i] < 0x20 || uri[i] == 0x7F) { err = true; break; }
  if (!err && n == 1 && uri[0] == '*') {
    t.single[S_REQUEST_URI] = {uri, 1};
  } else if (!err) {
    // getScheme
    uint32_t sn = 0, r0 = 0;
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t c = uri[i];
      if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) continue;
      if ((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.') {
        if (i == 0) break;
        continue;
      }
      if (c == ':') {
        if (i == 0) err = true;
        sn = i;
        r0 = i + 1;
      }
      break;
    }
    // rest = uri[r0, n): RawQuery (ForceQuery when the only '?' ends it)
    uint32_t nq = 0, q = n;
    for (uint32_t i = r0; i < n; i++)
      if (uri[i] == '?') {
        if (q == n) q = i;
        nq++;
      }
    const bool force_q = n > r0 && uri[n - 1] == '?' && nq == 1;
    const uint8_t* rest = uri + r0;
    uint32_t rn = q - r0;
    if (force_q) query = {uri + n, 0};
    else if (q < n) query = {uri + q + 1, n - q - 1};
    const uint32_t tail = (force_q || query.n) ? 1 + query.n : 0u;
    const uint8_t* hostp = nullptr;
    uint32_t hn = 0, un_ = 0;
    const uint8_t* userp = nullptr;  // userinfo (escaped form, String()) / its length
    bool has_user = false, omit_host = false, opaque = false, had_auth = false;
    if (!err && !(rn > 0 && rest[0] == '/')) {
      if (sn) {
        opaque = true;
      } else {
        for (uint32_t i = 0; i < rn && rest[i] != '/'; i++)
          if (rest[i] == ':') { err = true; break; }
      }
    }
    if (!err && !opaque) {
      if ((sn || !(rn >= 3 && rest[0] == '/' && rest[1] == '/' && rest[2] == '/')) && rn >= 2 && rest[0] == '/' &&
          rest[1] == '/') {
        had_auth = true;
        const uint8_t* au = rest + 2;
        uint32_t an = rn - 2;
        bool slash = false;
        for (uint32_t i = 0; i < an; i++)
          if (au[i] == '/') {
            rest = au + i;
            rn = an - i;
            an = i;
            slash = true;
            break;
          }
        if (!slash) {  // no '/' after the authority: the path is empty
          rest = au + an;
          rn = 0;
        }
        // parseAuthority: userinfo '@' host
        int64_t at = -1;
        for (uint32_t i = 0; i < an; i++)
          if (au[i] == '@') at = i;
        const uint8_t* h = at >= 0 ? au + at + 1 : au;
        const uint32_t hl = at >= 0 ? an - (uint32_t)at - 1 : an;
        // parseHost
        if (hl > 0 && h[0] == '[') {
          int64_t rb = -1;
          for (uint32_t i = 0; i < hl; i++)
            if (h[i] == ']') rb = i;
          if (rb < 0 || !valid_port(h + rb + 1, hl - (uint32_t)rb - 1)) err = true;
          for (uint32_t i = 0; !err && i + 2 < (uint32_t)rb; i++)
            if (h[i] == '%' && h[i + 1] == '2' && h[i + 2] == '5') {  // RFC 6874 zone: not restated
              t.flags |= GI_REQ_UNSUPPORTED_URI;
              return false;
            }
        } else {
          int64_t co = -1;
          for (uint32_t i = 0; i < hl; i++)
            if (h[i] == ':') co = i;
          if (co >= 0 && !valid_port(h + co, hl - (uint32_t)co)) err = true;
        }
        if (!err && !url_unescape_ok(h, hl, 1)) err = true;
        if (!err) {
          uint8_t* hd = tx_alloc(t, hl);
          if (!hd && hl) return false;
          hn = url_unescape(h, hl, hd);
          hostp = hd;
        }
        if (!err && at >= 0) {  // validUserinfo, then unescape + escape of user [":" password]
          const uint32_t ul = (uint32_t)at;
          for (uint32_t i = 0; i < ul && !err; i++) {
            const uint8_t c = au[i];
            bool okc = isalnum_(c);
            switch (c) {
              case '-': case '.': case '_': case ':': case '~': case '!': case '$': case '&': case '\'': case '(':
              case ')': case '*': case '+': case ',': case ';': case '=': case '%': case '@':
                okc = true;
            }
            if (!okc) err = true;
          }
          int64_t co = -1;
          for (uint32_t i = 0; i < ul && co < 0; i++)
            if (au[i] == ':') co = i;
          const uint32_t n1 = co >= 0 ? (uint32_t)co : ul;
          if (!err && (!url_unescape_ok(au, n1, 0) || (co >= 0 && !url_unescape_ok(au + co + 1, ul - n1 - 1, 0))))
            err = true;
          if (!err) {
            uint8_t* tmp = tx_alloc(t, ul);
            uint8_t* ue = tx_alloc(t, 3 * ul + 1);
            if ((!tmp && ul) || !ue) return false;
            uint32_t k = url_escape(tmp, url_unescape(au, n1, tmp), 2, ue);
            if (co >= 0) {
              ue[k++] = ':';
              const uint32_t m = url_unescape(au + co + 1, ul - n1 - 1, tmp);
              k += url_escape(tmp, m, 2, ue + k);
            }
            userp = ue;
            un_ = k;
            has_user = true;
          }
        }
      } else if (sn && rn > 0 && rest[0] == '/') {
        omit_host = true;
      }
    }
    if (!err && !opaque && !url_unescape_ok(rest, rn, 0)) err = true;
    if (!err) {
      // Path (decoded) and EscapedPath (the raw path when it encodes Path, else escape(Path))
      const uint8_t* p = rest;
      uint32_t pn = rn;
      bool has_pct = false;
      for (uint32_t i = 0; i < rn && !opaque; i++) has_pct |= rest[i] == '%';
      if (opaque) {
        p = rest;
        pn = 0;
      } else if (has_pct) {
        uint8_t* dp = tx_alloc(t, rn);
        if (!dp) return false;
        pn = url_unescape(rest, rn, dp);
        p = dp;
      }
      bool raw_ok = true;
      for (uint32_t i = 0; i < rn && !opaque; i++)
        if (!valid_encoded_path_char(rest[i])) { raw_ok = false; break; }
      uint32_t esc_len = 0;
      for (uint32_t i = 0; i < pn; i++) esc_len += should_escape_path(p[i]) ? 3 : 1;
      if (!raw_ok && !opaque && esc_len == rn) {  // escape(Path) == raw path
        raw_ok = true;
        uint32_t o = 0;
        const char* hx = "0123456789ABCDEF";
        for (uint32_t i = 0; i < pn && raw_ok; i++) {
          if (should_escape_path(p[i])) {
            raw_ok = rest[o] == '%' && rest[o + 1] == hx[p[i] >> 4] && rest[o + 2] == hx[p[i] & 15];
            o += 3;
          } else {
            raw_ok = rest[o] == p[i];
            o++;
          }
        }
      }
      const uint32_t en = opaque ? 0u : raw_ok ? rn : esc_len;
      if (!sn && !had_auth && raw_ok && !opaque) {
        // a path (origin-form) target: String() is the target itself (a
        // relative one with ':' in its first segment failed Parse above)
        t.single[S_REQUEST_URI] = {uri, n};
      } else {
        uint8_t* o = tx_alloc(t, sn + 1 + (opaque ? rn : 0) + 2 + un_ + 1 + 3 * hn + 3 + en + tail);
        if (!o) return false;
        uint32_t k = 0;
        for (uint32_t i = 0; i < sn; i++) o[k++] = alower(uri[i]);
        if (sn) o[k++] = ':';
        if (opaque) {
          for (uint32_t i = 0; i < rn; i++) o[k++] = rest[i];
        } else {
          if ((sn || hn || has_user) && !(omit_host && !hn && !has_user)) {
            if (hn || pn || has_user) {
              o[k++] = '/';
              o[k++] = '/';
            }
            if (has_user) {
              for (uint32_t i = 0; i < un_; i++) o[k++] = userp[i];
              o[k++] = '@';
            }
            k += url_escape(hostp, hn, 1, o + k);
          }
          if (en && (raw_ok ? rest[0] : (should_escape_path(p[0]) ? (uint8_t)'%' : p[0])) != '/' && hn) o[k++] = '/';
          if (k == 0) {  // a first segment with ':' would read as a scheme
            bool colon = false;
            for (uint32_t i = 0; i < pn && p[i] != '/'; i++) colon |= p[i] == ':';
            if (colon) {
              o[k++] = '.';
              o[k++] = '/';
            }
          }
          if (raw_ok) {
            for (uint32_t i = 0; i < rn; i++) o[k++] = rest[i];
          } else {
            k += url_escape(p, pn, 0, o + k);
          }
        }
        if (tail) {
          o[k++] = '?';
          for (uint32_t i = 0; i < query.n; i++) o[k++] = query.p[i];
        }
        t.single[S_REQUEST_URI] = {o, k};
      }
      parse_query(t, query.p, query.n, FK_ARG_GET);
      path = {p, pn};
    }
  }
  if (err) {
    t.single[S_REQUEST_URI] = {uri, n};
    path = {uri, n};
    query = {uri, 0};
  }
  t.single[S_REQUEST_FILENAME] = path;
  t.single[S_QUERY_STRING] = query;
  int64_t off = -1;
  for (uint32_t i = 0; i < path.n; i++)
    if (path.p[i] == '/') off = i;
  if (off != -1 && path.n > (uint32_t)off + 1)
    t.single[S_REQUEST_BASENAME] = {path.p + off + 1, path.n - (uint32_t)off - 1};
  else
    t.single[S_REQUEST_BASENAME] = path;
  return true;
}

GI_HD void parse_cookies(Tx& t, const uint8_t* v, uint32_t n) {
  uint32_t a = 0, e = n;
  while (a < e && isws(v[a])) a++;
  while (e > a && isws(v[e - 1])) e--;
  uint32_t i = a;
  while (i < e) {
    uint32_t j = i;
    while (j < e && v[j] != ';') j++;
    uint32_t pa = i, pe = j;
    while (pa < pe && isws(v[pa])) pa++;
    while (pe > pa && isws(v[pe - 1])) pe--;
    if (pe > pa) {
      uint32_t eq = pa;
      while (eq < pe && v[eq] != '=') eq++;
      if (eq < pe)
        add_field(t, FK_COOKIE, v + pa, eq - pa, v + eq + 1, pe - eq - 1);
      else
        add_field(t, FK_COOKIE, v + pa, pe - pa, v + pe, 0);
    }
    i = j + 1;
  }
}

GI_HD inline bool starts_ci(const uint8_t* s, uint32_t n, const char* lit) {
  uint32_t i = 0;
  for (; lit[i]; i++)
    if (i >= n || alower(s[i]) != (uint8_t)lit[i]) return false;
  return true;
}

GI_HD inline bool contains_ci(const uint8_t* s, uint32_t n, const char* lit) {
  for (uint32_t i = 0; i < n; i++)
    if (starts_ci(s + i, n - i, lit)) return true;
  return false;
}

// ------------------------------------------------------------ TX / macros
GI_HD __forceinline__ Str slot_str(Tx& t, const Slot& s, uint8_t* buf) {
  if (s.state == 1) return {buf, go_itoa(s.num, buf)};
  if (s.state == 2) return {s.p, s.n};
  return {buf, 0};
}
GI_HD __forceinline__ int64_t slot_int(const Slot& s, bool* ok) {
  if (s.state == 1) {
    *ok = true;
    return s.num;
  }
  if (s.state == 2) return go_atoi(s.p, s.n, ok);
  *ok = false;
  return 0;
}

// A single's value.  ARGS_COMBINED_SIZE is computed when read [upstream
// internal/collections/sized.go SizeCollection over ARGS_GET + ARGS_POST:
// the sum of len(key) + len(value) of every entry]; buf >= 24 bytes.
GI_HD __forceinline__ Str single_val(Tx& t, uint32_t sid, uint8_t* buf) {
  if (sid == S_ARGS_COMBINED_SIZE) {
    uint64_t n = 0;
    const uint32_t j0 = t.kx ? t.kx[FK_ARG_GET] : 0u, j1 = t.kx ? t.kx[FK_ARG_POST + 1] : t.nf;
    for (uint32_t j = j0; j < j1; j++) {
      const Field& fl = t.fields[t.kx ? t.kx[12 + j] : j];
      if (fl.kind == FK_ARG_GET || fl.kind == FK_ARG_POST) n += (uint64_t)fl.kn + fl.vn;
    }
    return {buf, go_itoa((int64_t)n, buf)};
  }
  return t.single[sid];
}

// Expand a %{..} template.  *persistent: result points into the program's
// string pool (safe to keep in TX); otherwise into the macro scratch.
GI_HD __forceinline__ Str expand(Tx& t, int32_t tid, bool* persistent) {
  const DProgram& P = *t.P;
  *persistent = false;
  if (tid < 0) return {t.mt, 0};
  const DTmpl tm = P.tmpls[tid];
  if (tm.part_count == 1 && P.tparts[tm.part_begin].kind == TP_LIT) {
    *persistent = true;
    const DTmplPart& p = P.tparts[tm.part_begin];
    return {P.strpool + p.off, p.len};
  }
  uint32_t o = 0;
  for (uint32_t k = 0; k < tm.part_count; k++) {
    const DTmplPart p = P.tparts[tm.part_begin + k];
    Str s{nullptr, 0};
    uint8_t nb[24];
    if (p.kind == TP_LIT) {
      s = {P.strpool + p.off, p.len};
    } else if (p.kind == TP_TX) {
      const Slot sv = slot_rd(t, (uint32_t)p.slot);
      s = slot_str(t, sv, nb);
    } else if (p.kind == TP_SINGLE) {
      s = single_val(t, p.single, nb);
    } else if (p.kind == TP_MV) {
      if (t.mv) s = {mv_curval(t.mv), t.mv->cur_vn};  // (no state: an unreachable rule, compile.cpp dead)
    } else if (p.kind == TP_MVNAME) {
      if (t.mv) s = {mv_curname(t.mv), t.mv->cur_nn};
    } else if (p.kind == TP_HEADER) {
      for (uint32_t f = 0; f < t.nf; f++)
        if (t.fields[f].kind == FK_HEADER && eq_ascii_ci(t.fields[f].k, t.fields[f].kn, P.strpool + p.off, p.len)) {
          s = {t.fields[f].v, t.fields[f].vn};
          break;
        }
    }
    if (o + s.n > t.cap_mt) {
      t.flags |= GI_REQ_OVERFLOW;
      return {t.mt, 0};
    }
    copy_bytes(t.mt + o, s.p, s.n);
    o += s.n;
  }
  return {t.mt, o};
}

// Run-time TX keys (setvar:'tx.header_name_920450_%{tx.0}=...'): the request's
// dynamic area holds DynHdr, then cap DynEnt records (in creation order), then
// capb bytes for their keys and string values.  runtime.cpp sizes it from the
// request (DDynSite), so it never runs out; a full area still only flags
// GI_REQ_OVERFLOW.
struct DynHdr {
  uint32_t n, cap, nb, capb;
};
struct DynEnt {
  const uint8_t* k;
  uint32_t kn, h;
  Slot s;
};
static_assert(sizeof(DynEnt) == 32, "runtime.cpp sizes DynEnt as 32 bytes");
GI_HD __forceinline__ DynEnt* dyn_ents(uint8_t* d) { return (DynEnt*)(d + sizeof(DynHdr)); }
GI_HD __forceinline__ uint8_t* dyn_alloc(uint8_t* d, uint32_t n) {
  DynHdr* H = (DynHdr*)d;
  if (H->nb + n > H->capb) return nullptr;
  uint8_t* p = d + sizeof(DynHdr) + 32ull * H->cap + H->nb;
  H->nb += n;
  return p;
}

// The slot of a macro-key setvar, given its expanded key in kp (lowercased
// here) [upstream setvar.go: strings.ToLower of the expanded key; ASCII, like
// the compiler's static TX names]: a key that names a static slot returns
// *sid = that slot; otherwise the dynamic entry with that key (created unless
// delete).  *ovf: the area is full.  No Tx& parameter: a non-inlined callee
// taking the Tx by reference would force k_eval's Tx out of registers.
GI_HD __noinline__ Slot* dyn_lookup(const DProgram& P, uint8_t* dyn, uint8_t* kp, uint32_t kn, bool create,
                                    int32_t* sid, bool* ovf) {
  copy_lower(kp, kp, kn);
  const uint32_t h = fnv1a_w(kp, kn);
  for (uint32_t i = h & P.slot_hash_mask;; i = (i + 1) & P.slot_hash_mask) {
    const uint32_t e = P.slot_hash[i];
    if (!e) break;
    if (eq_bytes_w(P.strpool + P.slot_names[2 * (e - 1)], P.slot_names[2 * (e - 1) + 1], kp, kn)) {
      *sid = (int32_t)(e - 1);
      return nullptr;
    }
  }
  DynHdr* H = (DynHdr*)dyn;
  DynEnt* E = dyn_ents(dyn);
  for (uint32_t j = 0; j < H->n; j++)
    if (E[j].h == h && eq_bytes_w(E[j].k, E[j].kn, kp, kn)) return &E[j].s;
  if (!create) return nullptr;
  uint8_t* kb = H->n < H->cap ? dyn_alloc(dyn, kn) : nullptr;
  if (!kb) {
    *ovf = true;
    return nullptr;
  }
  copy_bytes(kb, kp, kn);
  DynEnt& ne = E[H->n++];
  ne.k = kb;
  ne.kn = kn;
  ne.h = h;
  ne.s.num = 0;
  ne.s.n = 0;
  ne.s.state = 0;
  return &ne.s;
}

// setvar [upstream internal/actions/setvar.go]
GI_HD __forceinline__ void run_setvar(Tx& t, const DAction& a) {
  Slot* slp;
  if (a.slot >= 0) {
    slp = &slot_wr(t, (uint32_t)a.slot);
  } else {  // a key with a macro: expanded into the macro scratch, then looked up
    bool kpers;
    const Str k = expand(t, a.aux, &kpers);
    if (t.flags & GI_REQ_OVERFLOW) return;
    int32_t sid = -1;
    bool ovf = false;
    slp = dyn_lookup(*t.P, t.dyn, (uint8_t*)k.p, k.n, a.kind == A_SETVAR, &sid, &ovf);
    if (ovf) {
      t.flags |= GI_REQ_OVERFLOW;
      return;
    }
    if (sid >= 0) slp = &slot_wr(t, (uint32_t)sid);
  }
  if (!slp) return;
  Slot& sl = *slp;
  if (a.kind == A_SETVAR_DEL) {
    sl.state = 0;
    return;
  }
  // fast forms: same results as the expanding path below, without strings
  if (a.a == SV_SET_INT) {
    sl.state = 1;
    sl.num = a.b;
    return;
  }
  if (a.a != SV_GENERIC) {
    int64_t vv = a.b;
    if (a.a == SV_ADD_SLOT || a.a == SV_SUB_SLOT) {
      const Slot src = slot_rd(t, (uint32_t)a.b);
      if (src.state == 0) return;  // "+" alone: Atoi("") fails, no change
      if (src.state != 1) goto generic;
      vv = src.num;
    }
    {
      bool ok;
      int64_t me = slot_int(sl, &ok);
      if (!ok) me = 0;
      const bool add = a.a == SV_ADD_CONST || a.a == SV_ADD_SLOT;
      sl.state = 1;
      sl.num = (int64_t)(add ? (uint64_t)me + (uint64_t)vv : (uint64_t)me - (uint64_t)vv);
      return;
    }
  }
generic:
  bool pers;
  Str v = expand(t, a.tmpl, &pers);
  if (v.n == 0) {
    sl.state = 2;
    sl.p = v.p;
    sl.n = 0;
    return;
  }
  if (v.p[0] == '+' || v.p[0] == '-') {
    bool ok;
    int64_t me = slot_int(sl, &ok);
    if (!ok) me = 0;
    int64_t vv = go_atoi(v.p + 1, v.n - 1, &ok);
    if (!ok) return;
    uint64_t r = v.p[0] == '+' ? (uint64_t)me + (uint64_t)vv : (uint64_t)me - (uint64_t)vv;
    sl.state = 1;
    sl.num = (int64_t)r;
    return;
  }
  // canonical decimal -> keep as integer
  bool ok;
  int64_t num = go_atoi(v.p, v.n, &ok);
  if (ok) {
    uint8_t buf[24];
    uint32_t k = go_itoa(num, buf);
    if (eq_bytes(buf, k, v.p, v.n)) {
      sl.state = 1;
      sl.num = num;
      return;
    }
  }
  if (pers) {
    sl.state = 2;
    sl.p = v.p;
    sl.n = v.n;
    return;
  }
  uint8_t* dst;
  if (a.slot < 0) {  // a run-time key: its value lives in the dynamic area the host sized for it
    dst = dyn_alloc(t.dyn, v.n);
    if (!dst) {
      t.flags |= GI_REQ_OVERFLOW;
      return;
    }
  } else {
    if (t.ntx + v.n > t.cap_tx) {
      t.flags |= GI_REQ_OVERFLOW;
      return;
    }
    dst = t.txa + t.ntx;
    t.ntx += v.n;
  }
  copy_bytes(dst, v.p, v.n);
  sl.state = 2;
  sl.p = dst;
  sl.n = v.n;
}

GI_HD __forceinline__ void run_actions(Tx& t, const DRule& R) {
  const DProgram& P = *t.P;
  const uint64_t c0 = t.profon ? gi_clock() : 0;
  struct ProfEnd {
    Tx& t;
    uint64_t c0;
    GI_HD ~ProfEnd() {
      if (t.profon) t.prof_act_cyc += gi_clock() - c0;
    }
  } prof_end{t, c0};
  for (uint32_t k = 0; k < R.act_count; k++) {
    const DAction a = gi_cload(P.acts, R.act_begin + k);
    switch (a.kind) {
      case A_SETVAR:
      case A_SETVAR_DEL:
        run_setvar(t, a);
        break;
      case A_CTL_RULE_REMOVE_ID:
        if (t.nremoved < 8) {
          t.removed[t.nremoved][0] = a.a;
          t.removed[t.nremoved][1] = a.b;
          t.nremoved++;
        } else {
          t.flags |= GI_REQ_OVERFLOW;
        }
        break;
      case A_CTL_RULE_REMOVE_TARGET:
        if (t.nrtgt < 8) {
          t.rtgt[t.nrtgt] = {a.a, a.b, (uint32_t)a.slot, (uint32_t)a.tmpl, (uint32_t)a.aux, 0u};
          t.nrtgt++;
        } else {
          t.flags |= GI_REQ_OVERFLOW;
        }
        break;
      case A_CTL_RULE_REMOVE_GROUP:
        t.rm_groups |= 1u << (uint32_t)a.a;
        break;
      case A_CTL_RULE_ENGINE:
        t.engine = (uint8_t)a.a;
        break;
      case A_CTL_BODY_PROCESSOR: {
        t.body_proc = (uint8_t)a.a;
        const uint8_t* s = a.a == BP_URLENCODED ? CS_URLENCODED : a.a == BP_JSON ? CS_JSON
                           : a.a == BP_XML ? CS_XML : CS_MULTIPART;
        uint32_t n = a.a == BP_URLENCODED ? 10 : a.a == BP_JSON ? 4 : a.a == BP_XML ? 3 : 9;
        t.single[S_REQBODY_PROCESSOR] = {s, n};
        break;
      }
      case A_CTL_BODY_ACCESS:
        t.body_access = (uint8_t)a.a;
        break;
      case A_CTL_FORCE_BODY:
        t.force_body = (uint8_t)a.a;
        break;
    }
  }
}

// ------------------------------------------------------------- operators
// Go net.ParseIP (compile.cpp go_parse_ip) + IP.To4: *n = 4 (IPv4, or an
// IPv4-mapped IPv6 address) or 16.
GI_HD bool dev_parse_ipv4(const uint8_t* s, uint32_t len, uint8_t* out) {
  uint32_t i = 0;
  for (int f = 0; f < 4; f++) {
    if (f) {
      if (i >= len || s[i] != '.') return false;
      i++;
    }
    uint32_t j = i, v = 0;
    while (j < len && j - i < 3 && s[j] >= '0' && s[j] <= '9') v = v * 10 + (s[j++] - '0');
    if (j == i || v > 255 || (j - i > 1 && s[i] == '0')) return false;
    out[f] = (uint8_t)v;
    i = j;
  }
  return i == len;
}
GI_HD bool dev_parse_ip(const uint8_t* s, uint32_t len, uint8_t* out, uint32_t* n) {
  bool colon = false;
  for (uint32_t i = 0; i < len; i++) {
    if (s[i] == ':') colon = true;
    if (s[i] == '%') return false;
  }
  if (!colon) {
    *n = 4;
    return dev_parse_ipv4(s, len, out);
  }
  uint16_t g[8];
  int ng = 0, gap = -1;
  uint32_t i = 0;
  if (len >= 2 && s[0] == ':' && s[1] == ':') {
    gap = 0;
    i = 2;
  }
  while (i < len) {
    if (ng == 8) return false;
    uint32_t j = i, v = 0;
    while (j < len && j - i < 4 && ishex(s[j])) v = v * 16 + hexv(s[j++]);
    if (j < len && s[j] == '.') {
      uint8_t v4[4];
      if (ng > 6 || !dev_parse_ipv4(s + i, len - i, v4)) return false;
      g[ng++] = (uint16_t)(v4[0] << 8 | v4[1]);
      g[ng++] = (uint16_t)(v4[2] << 8 | v4[3]);
      i = len;
      break;
    }
    if (j == i) return false;
    g[ng++] = (uint16_t)v;
    i = j;
    if (i == len) break;
    if (s[i] != ':') return false;
    i++;
    if (i < len && s[i] == ':') {
      if (gap >= 0) return false;
      gap = ng;
      i++;
      if (i == len) break;
    } else if (i == len) {
      return false;
    }
  }
  if ((gap < 0 && ng != 8) || (gap >= 0 && ng > 7)) return false;
  uint16_t full[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (gap < 0) {
    for (int k = 0; k < 8; k++) full[k] = g[k];
  } else {
    for (int k = 0; k < gap; k++) full[k] = g[k];
    for (int k = 0; k < ng - gap; k++) full[8 - (ng - gap) + k] = g[gap + k];
  }
  const bool mapped = !full[0] && !full[1] && !full[2] && !full[3] && !full[4] && full[5] == 0xFFFF;
  if (mapped) {  // IP.To4
    out[0] = (uint8_t)(full[6] >> 8); out[1] = (uint8_t)full[6];
    out[2] = (uint8_t)(full[7] >> 8); out[3] = (uint8_t)full[7];
    *n = 4;
    return true;
  }
  for (int k = 0; k < 8; k++) {
    out[2 * k] = (uint8_t)(full[k] >> 8);
    out[2 * k + 1] = (uint8_t)full[k];
  }
  *n = 16;
  return true;
}

// coraza ipmatch.go Evaluate: net.ParseIP(value), then IPNet.Contains per network.
GI_HD bool ip_match(const uint8_t* recs, uint32_t rlen, const uint8_t* s, uint32_t n) {
  uint8_t ip[16];
  uint32_t fam;
  if (!dev_parse_ip(s, n, ip, &fam)) return false;
  for (uint32_t r = 0; r + GI_IPNET_BYTES <= rlen; r += GI_IPNET_BYTES) {
    const uint8_t* rec = recs + r;
    if (rec[0] != fam) continue;
    uint32_t bits = rec[1];
    bool ok = true;
    for (uint32_t k = 0; k < fam && bits && ok; k++) {
      const uint32_t keep = bits >= 8 ? 8u : bits;
      const uint8_t m = (uint8_t)(0xFF00u >> keep);
      ok = (ip[k] & m) == rec[2 + k];
      bits -= keep;
    }
    if (ok) return true;
  }
  return false;
}

GI_HD bool contains_word(const uint8_t* v, uint32_t vn, const uint8_t* w, uint32_t wn) {
  if (wn == 0) return true;
  for (uint32_t i = 0; i + wn <= vn; i++) {
    uint32_t k = 0;
    while (k < wn && v[i + k] == w[k]) k++;
    if (k < wn) continue;
    bool before = i == 0 || !(isalnum_(v[i - 1]) || v[i - 1] == '_');
    uint32_t j = i + wn;
    bool after = j >= vn || !(isalnum_(v[j]) || v[j] == '_');
    if (before && after) return true;
  }
  return false;
}

// DETECT = false (k_body): @detectSQLi/@detectXSS cannot reach the call (the
// compiler keeps REQUEST_BODY detect links out of k_body), so the kernel does
// not link libinjection and keeps its register budget.
template <bool DETECT = true>
GI_HD __forceinline__ bool eval_op(Tx& t, const DOp& o, const uint8_t* s, uint32_t n) {
  const DProgram& P = *t.P;
  bool res = false;
  switch (o.kind) {
    case OP_RX:
    case OP_PM:
      res = o.nfa >= 0 ? nfa_match(P, o.nfa, s, n) : dfa_match(P, o.dfa, s, n, false);
      for (uint32_t g = 1; g < o.ngroups && !res; g++) res = dfa_match(P, o.dfa + (int32_t)g, s, n, false);
      break;
    case OP_UNCONDITIONAL:
      res = true;
      break;
    case OP_IPMATCH:
      res = ip_match(P.strpool + o.lit_off, o.lit_len, s, n);
      break;
    case OP_NOMATCH:
      res = false;
      break;
    case OP_DETECT_SQLI:  // [upstream] detect_sqli.go: libinjection.IsSQLi (capture of the fingerprint is unobservable here)
      if (DETECT) {
        // the tokenizer state of this lane in LDS (k_eval's 128-thread blocks;
        // k_eval_wave's lanes run identical copies): every state access is an
        // LDS access instead of a round trip to the request's HBM scratch
#if defined(__HIP_DEVICE_COMPILE__)
        __shared__ LiSqli li_st[128];
        res = li_detect_sqli(s, n, &li_st[threadIdx.x & 127u], li_tables_const());
#else
        LiSqli li_st;  // the host interpreter: a stack copy
        res = li_detect_sqli(s, n, &li_st, li_tables_const());
#endif
      }
      break;
    case OP_DETECT_XSS:  // detect_xss.go: libinjection.IsXSS
      if (DETECT) res = li_detect_xss(s, n);
      break;
    case OP_VALIDATE_BYTE_RANGE:
      for (uint32_t i = 0; i < n; i++)
        if (!((o.bits[s[i] >> 5] >> (s[i] & 31)) & 1)) { res = true; break; }
      break;
    case OP_VALIDATE_URL_ENCODING:
      for (uint32_t i = 0; i < n;) {
        if (s[i] == '%') {
          if (i + 2 >= n) { res = true; break; }
          if (ishex(s[i + 1]) && ishex(s[i + 2])) i += 3;
          else { res = true; break; }
        } else {
          i++;
        }
      }
      break;
    case OP_VALIDATE_UTF8:
      for (uint32_t i = 0; i < n;) {
        uint32_t w;
        uint32_t r = decode_rune(s, n, i, &w);
        if (r == 0xFFFD && w == 1) { res = true; break; }
        i += w;
      }
      break;
    case OP_EQ: case OP_GE: case OP_GT: case OP_LE: case OP_LT: {
      int64_t a;
      bool ok;
      if (o.has_num) {
        a = o.num;
      } else {
        bool pers;
        Str x = expand(t, o.tmpl, &pers);
        a = go_atoi(x.p, x.n, &ok);
        if (!ok) a = 0;
      }
      int64_t b = go_atoi(s, n, &ok);
      if (!ok) b = 0;
      res = o.kind == OP_EQ ? b == a : o.kind == OP_GE ? b >= a : o.kind == OP_GT ? b > a
            : o.kind == OP_LE ? b <= a : b < a;
      break;
    }
    default: {
      Str a;
      if (o.arg_is_lit) {
        a = {P.strpool + o.lit_off, o.lit_len};
      } else {
        bool pers;
        a = expand(t, o.tmpl, &pers);
      }
      switch (o.kind) {
        case OP_CONTAINS:
          res = (o.arg_is_lit && o.dfa >= 0) ? dfa_match(P, o.dfa, s, n, false) : find_bytes(s, n, a.p, a.n) >= 0;
          break;
        case OP_CONTAINSWORD: res = contains_word(s, n, a.p, a.n); break;
        case OP_STREQ: res = eq_bytes(s, n, a.p, a.n); break;
        case OP_BEGINSWITH: res = n >= a.n && eq_bytes(s, a.n, a.p, a.n); break;
        case OP_ENDSWITH: res = n >= a.n && eq_bytes(s + n - a.n, a.n, a.p, a.n); break;
        case OP_WITHIN:
          if (o.arg_is_lit && o.dfa >= 0) {  // the argument's suffix automaton (compile.cpp within_dfa)
            const DDfa d = gi_cload(P.dfas, (uint64_t)o.dfa);
            const uint16_t* tr = P.trans + d.trans_off;
            const uint8_t* am = P.u8pool + d.amap_off;
            uint32_t st = d.start;
            for (uint32_t i = 0; i < n && st != d.accept; i++) st = tr[st * d.n_classes + am[s[i]]];
            res = st != d.accept;
          } else {
            res = find_bytes(a.p, a.n, s, n) >= 0;
          }
          break;
      }
    }
  }
  return o.negate ? !res : res;
}

// Exact hit set (k_eval's per-value phase-A results): a key per (hit slot,
// value index) records that this value, transformed by the link's chain,
// satisfies the link's operator (maybe = 0), or that phase A could not decide
// it (maybe = 1: chain overflow, list overflow).  A value of a value-exact
// slot with neither key cannot match the link.  Keys need slot < 65535 and
// vix < 32768; a request with a key outside that range, or whose table fills,
// gets the overflow word set and k_eval re-evaluates as without the set.
GI_HD __forceinline__ uint32_t hset_key(uint32_t slot, uint32_t vix, uint32_t maybe) {
  return ((slot + 1u) << 16) | (vix << 1) | maybe;
}
GI_HD __forceinline__ uint32_t hset_hash(uint32_t k) {
  k ^= k >> 15;
  k *= 0x2C1B3C6Du;
  k ^= k >> 12;
  return k;
}
__device__ __noinline__ void hset_insert(const DBatch& B, const ReqLayout& L, uint32_t slot, uint32_t vix, uint32_t maybe) {
  uint32_t* tab = B.hset + L.hset_word;
  if (slot >= 65534u || vix >= 32768u) {
    tab[0] = 1u;
    return;
  }
  const uint32_t key = hset_key(slot, vix, maybe);
  uint32_t h = hset_hash(key) & L.hset_mask;
  for (uint32_t probe = 0; probe <= L.hset_mask; probe++) {
    const uint32_t prev = atomicCAS(&tab[1 + h], 0u, key);
    if (prev == 0u || prev == key) return;
    h = (h + 1) & L.hset_mask;
  }
  tab[0] = 1u;  // full
}
// k_eval: 0 = no key, 1 = exact match, 2 = maybe (evaluate the value)
GI_HD __forceinline__ uint32_t hset_lookup(const uint32_t* tab, uint32_t mask, uint32_t slot, uint32_t vix) {
  uint32_t res = 0;
  for (uint32_t m = 0; m < 2 && !res; m++) {
    const uint32_t key = hset_key(slot, vix, m);
    uint32_t h = hset_hash(key) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++) {
      const uint32_t x = tab[1 + h];
      if (x == key) {
        res = 1 + m;
        break;
      }
      if (x == 0u) break;
      h = (h + 1) & mask;
    }
  }
  return res;
}

// ------------------------------------------------------------ captures
// Header of the per-request capture workspace (k_eval sets it up), then the
// pike_match workspace.
#define GI_CAPWS_HDR 16
struct CapHdr {
  uint32_t nrec, nbytes;     // records / bytes written for this request
  uint32_t* rec;             // its row of gi_capture records (4 words each)
  uint8_t* bytes;            // its row of capture bytes
  uint32_t rec_cap, bytes_cap;
  uint32_t trunc;            // records or bytes did not fit
  uint32_t _pad[7];
};
static_assert(sizeof(CapHdr) == 4 * GI_CAPWS_HDR, "CapHdr layout");

// [upstream rx.go Evaluate, capturing]: FindStringSubmatch(value); groups
// 0..8 -> TX.0..TX.8 (transaction.go CaptureField: TX SetIndex(strconv.Itoa(i)),
// unset groups ""), each value copied into its group's buffer; one capture
// record per group.  Returns GI_REQ_OVERFLOW when the value does not fit.
GI_HD __noinline__ uint32_t run_capture(const DProgram& P, uint32_t* capws, uint8_t* capbuf, uint32_t cap_t,
                                             Slot* slots, uint32_t n_req, uint32_t rule_id, int32_t pike,
                                             const uint8_t* v, uint32_t n) {
  const DPike pk = P.pikes[pike];
  int32_t caps[GI_PIKE_MAX_SLOTS];
  CapHdr* H = (CapHdr*)capws;
  if (pk.whole) {  // (?sm)^.*$: the whole value, without running the VM
    caps[0] = 0;
    caps[1] = (int32_t)n;
  } else if (!pike_match(P.pike_insts + pk.inst_off, P.pike_ranges, pk, v, n, capws + GI_CAPWS_HDR, caps)) {
    return 0;
  }
  if (n > cap_t) return GI_REQ_OVERFLOW;
  const uint32_t stride = (cap_t + 15) & ~15u;
  for (uint32_t g = 0; 2 * g < pk.nslot && g < 9; g++) {
    const int32_t a = caps[2 * g], b = caps[2 * g + 1];
    const uint32_t len = (a >= 0 && b >= a) ? (uint32_t)(b - a) : 0u;
    uint8_t* dst = capbuf + (uint64_t)g * stride;
    copy_bytes(dst, v + a, len);
    const int32_t sl = P.cap_slots[g];
    if (sl >= 0) {
      Slot& x = slots[(uint64_t)sl * n_req];
      x.state = 2;
      x.p = dst;
      x.n = len;
    }
    if (H->rec) {  // capture record {rule id, group, byte offset in the request's row, length}
      // (the first record that does not fit ends the list: the records kept
      // are a prefix of Coraza's, which GI_REQ_CAPTURE_TRUNC promises)
      if (!H->trunc && H->nrec < H->rec_cap && H->nbytes + len <= H->bytes_cap) {
        uint32_t* r = H->rec + 4ull * H->nrec;
        r[0] = rule_id;
        r[1] = g;
        r[2] = H->nbytes;
        r[3] = len;
        copy_bytes(H->bytes + H->nbytes, dst, len);
        H->nbytes += len;
        H->nrec++;
      } else {
        H->trunc = 1;
      }
    }
  }
  return 0;
}

// ------------------------------------------------------------ evaluation
// Apply the rule's transformation chain; returns the value to test.
GI_HD __forceinline__ Str transform(Tx& t, const DRule& R, const uint8_t* v, uint32_t vn, bool* ok,
                                       uint32_t kmax = 0xffffffffu) {
  const DProgram& P = *t.P;
  Str cur{v, vn};
  *ok = true;
  const uint32_t kn = min(kmax, R.tchain_len);
  uint32_t summ = kn ? value_summary(v, vn) : 0u;
  for (uint32_t k = 0; k < kn; k++) {
    const uint8_t code = P.tchains[R.tchain_off + k];
    if (transform_identity(summ, code)) continue;  // identity on this value
    uint8_t* dst = (cur.p == t.t0) ? t.t1 : t.t0;
    int64_t m = apply_transform(P, code, cur.p, cur.n, dst, t.cap_t);
    if (m < 0) {
      t.flags |= GI_REQ_OVERFLOW;
      *ok = false;
      return {dst, 0};
    }
    cur = {dst, (uint32_t)m};
    summ = value_summary(cur.p, cur.n);
  }
  return cur;
}

// ctl:ruleRemoveTargetById: the link's rule id removed variable `var`
// entries with key k (coraza rule.go doEvaluate adds them to the variable's
// exceptions: compared with the lowercased key; a single's key is "")
// (ctl:ruleRemoveTargetByTag / ByMsg entries name a removal group: the rule's
// groups `groups` must hold it)
GI_HD __noinline__ bool target_removed_in(const Tx::RmTarget* rt, uint32_t n, const uint8_t* strpool, int32_t id,
                                               uint32_t groups, uint32_t var, const uint8_t* k, uint32_t kn) {
  for (uint32_t e = 0; e < n; e++) {
    const Tx::RmTarget x = rt[e];
    const bool sel = x.lo == GI_RM_GROUP_MODE ? ((groups >> (uint32_t)x.hi) & 1u) != 0u : (x.lo <= id && id <= x.hi);
    if (x.var == var && sel && eq_ascii_ci(k, kn, strpool + x.koff, x.klen)) return true;
  }
  return false;
}
#define target_removed(t, id, var, k, kn) \
  target_removed_in((t).rtgt, (t).nrtgt, (t).P->strpool, (id), (t).cur_groups, (var), (k), (kn))

// The link's phase-A bits are void: it can see ARGS_POST / body fields phase A
// did not scan for it (the gate's first stage scans the speculative parser's
// body fields only through the prefix streams, so there a RF2_PREFIX link's
// bits stay valid -- but not when the interpreter parsed the body itself:
// a processor phase 1 chose differently, a ProcessPartial body over the
// limit; phase A never saw those fields).
GI_HD __forceinline__ bool bodydep_void(const Tx& t, const DRule& R) {
  return (R.flags & RF_BODYDEP) && t.has_post && !(t.prefix_spec && (R.flags2 & RF2_PREFIX));
}

// A clear hit bit does not settle the link: some residual target (a mutable
// single, or a body collection the request actually has) is still to test.
GI_HD __forceinline__ bool residual_live(const Tx& t, const DRule& R) {
  if (!(R.flags & RF_RESIDUAL) || t.rcoll) return (R.flags & RF_RESIDUAL) != 0;
  return !(R.flags2 & RF2_RESID_COLL) && !((R.flags2 & RF2_RESID_RB) && !t.rbody);
}

GI_HD __forceinline__ bool key_excluded(Tx& t, const DVarRef& vr, const uint8_t* k, uint32_t kn) {
  const DProgram& P = *t.P;
  for (uint32_t e = 0; e < vr.exc_count; e++) {
    const DExc x = P.excs[vr.exc_begin + e];
    if (x.dfa >= 0) {
      if (dfa_match(P, x.dfa, k, kn, true)) return true;
    } else if (eq_ascii_ci(k, kn, P.strpool + x.off, x.len)) {
      return true;
    }
  }
  return false;
}

GI_HD inline bool field_in(uint8_t var, uint32_t kind, bool* names) {
  *names = false;
  switch (var) {
    case V_ARGS_GET: return kind == FK_ARG_GET;
    case V_ARGS_POST: return kind == FK_ARG_POST;
    case V_ARGS: return kind == FK_ARG_GET || kind == FK_ARG_POST;
    case V_REQUEST_HEADERS: return kind == FK_HEADER;
    case V_REQUEST_COOKIES: return kind == FK_COOKIE;
    case V_ARGS_GET_NAMES: *names = true; return kind == FK_ARG_GET;
    case V_ARGS_POST_NAMES: *names = true; return kind == FK_ARG_POST;
    case V_ARGS_NAMES: *names = true; return kind == FK_ARG_GET || kind == FK_ARG_POST;
    case V_REQUEST_HEADERS_NAMES: *names = true; return kind == FK_HEADER;
    case V_REQUEST_COOKIES_NAMES: *names = true; return kind == FK_COOKIE;
    case V_FILES: return kind == FK_FILE;
    case V_FILES_NAMES: return kind == FK_FILE_NAME;
    case V_FILES_SIZES: return kind == FK_FILE_SIZE;
    case V_MULTIPART_PART_HEADERS: return kind == FK_PART_HEADER;
    case V_XML: return kind == FK_XML;
  }
  return false;
}

// The field kinds a collection reads (field_in), as the range [*lo, *hi]
// (empty: *lo > *hi).  Every collection's kinds are contiguous.
GI_HD __forceinline__ void var_kinds(uint8_t var, uint32_t* lo, uint32_t* hi) {
  uint32_t a = 1, b = 0;
  switch (var) {
    case V_ARGS_GET: case V_ARGS_GET_NAMES: a = b = FK_ARG_GET; break;
    case V_ARGS_POST: case V_ARGS_POST_NAMES: a = b = FK_ARG_POST; break;
    case V_ARGS: case V_ARGS_NAMES: a = FK_ARG_GET; b = FK_ARG_POST; break;
    case V_REQUEST_HEADERS: case V_REQUEST_HEADERS_NAMES: a = b = FK_HEADER; break;
    case V_REQUEST_COOKIES: case V_REQUEST_COOKIES_NAMES: a = b = FK_COOKIE; break;
    case V_FILES: a = b = FK_FILE; break;
    case V_FILES_NAMES: a = b = FK_FILE_NAME; break;
    case V_FILES_SIZES: a = b = FK_FILE_SIZE; break;
    case V_MULTIPART_PART_HEADERS: a = b = FK_PART_HEADER; break;
    case V_XML: a = b = FK_XML; break;
  }
  *lo = a;
  *hi = b;
}

// The fields grouped by kind, in the request arena: kx[k] is where kind k
// starts in the list kx + 12 (kx[10]: its length), each kind in field
// order.  A collection then visits only its own fields (in the order a scan
// of all fields would: ARGS' two kinds are GET args, then POST args, and every
// GET arg precedes every POST arg).  Rebuilt when a body parse adds fields;
// an arena without room leaves kx null (scan every field).
// (nb by value, the arena bytes it used returned in kx[11]: a pointer into the
// caller's Tx would pin the whole Tx in scratch memory)
GI_HD __noinline__ const uint32_t* build_kindex(const Field* fields, uint32_t nf, uint8_t* bytes, uint32_t nb,
                                                    uint32_t cap_b) {
  const uint32_t pad = (4u - (uint32_t)((uintptr_t)(bytes + nb) & 3u)) & 3u;
  if ((uint64_t)nb + pad + 4ull * (12ull + nf) > cap_b) return nullptr;
  uint32_t* kx = (uint32_t*)(bytes + nb + pad);
  for (uint32_t k = 0; k < 12; k++) kx[k] = 0;
  for (uint32_t f = 0; f < nf; f++) kx[min((uint32_t)fields[f].kind, 9u) + 1]++;
  for (uint32_t k = 1; k <= 10; k++) kx[k] += kx[k - 1];
  for (uint32_t f = 0; f < nf; f++) kx[12 + kx[min((uint32_t)fields[f].kind, 9u)]++] = f;
  for (uint32_t k = 10; k >= 1; k--) kx[k] = kx[k - 1];
  kx[0] = 0;
  kx[11] = pad + 4u * (12u + nf);
  return kx;
}
GI_HD __forceinline__ const uint32_t* kindex_into(const Field* fields, uint32_t nf, uint8_t* bytes, uint32_t& nb,
                                                  uint32_t cap_b) {
  const uint32_t* kx = build_kindex(fields, nf, bytes, nb, cap_b);
  if (kx) nb += kx[11];
  return kx;
}

// Test one value: transform, operator, per-match actions.  Returns the number of matches.
// multiMatch (coraza internal/corazawaf/rule.go executeTransformationsMultimatch):
// the operator runs on the untransformed value and again after each
// transformation of the chain that changed the value (an unchanged step adds
// no candidate); every match counts and runs the actions.  One eval_op /
// run_actions site serves both forms (the Tx stays in registers).
// var / k / kn name the value for the matched-variable state (MATCHED_VAR_NAME = VAR[:key]).
// exact (non-multiMatch links): phase A proved the transformed value matches
// (k_eval's hit set): the operator does not run again, and the chain runs
// only when the matched-variable state needs the transformed value.
GI_HD __forceinline__ uint32_t test_value(Tx& t, const DRule& R, const DOp& o, const uint8_t* v, uint32_t vn,
                                               uint32_t var, const uint8_t* key, uint32_t kn, bool exact = false) {
  uint32_t nm = 0;
  const uint8_t* cp = v;  // current candidate
  uint32_t cn = vn;
  uint32_t k = 0;         // transformations applied so far
  if (!(R.flags & RF_MULTIMATCH)) {
    if (!exact || t.mv || (R.flags & RF_CAPTURE)) {
      bool ok;
      const Str tv = transform(t, R, v, vn, &ok);
      if (!ok) return 0;
      cp = tv.p;
      cn = tv.n;
    }
    k = R.tchain_len;
  }
  // `fresh` = cp is a candidate not yet tested.  The loop body has no
  // continue: a candidate search written with continue/break was
  // miscompiled here (a lane's candidate update after an early loop exit was
  // lost while other lanes of the wave took the identity path).
  for (bool fresh = true;; k++) {
    if (fresh) {
      if (t.profon && !exact) t.prof_ops++;
      const bool hit = exact || eval_op(t, o, cp, cn);
      // capturing @rx: a value the regex matches writes TX.0-TX.8 -- for a
      // negated operator exactly the values that do not make the link match
      if ((R.flags & RF_CAPTURE) && hit != (o.negate != 0))
        t.flags |= run_capture(*t.P, t.capws, t.capbuf, t.cap_t, t.slots, t.n_req, t.cur_id, o.pike, cp, cn);
      if (hit) {
        if (t.mv && !mv_record(t.mv, var, key, kn, cp, cn)) t.flags |= GI_REQ_OVERFLOW;
        run_actions(t, R);
        nm++;
      }
    }
    if (k >= R.tchain_len) break;
    const uint8_t code = t.P->tchains[R.tchain_off + k];
    bool changed = false;
    if (!transform_identity(value_summary(cp, cn), code)) {  // else an identity on cp
      uint8_t* dst = (cp == t.t0) ? t.t1 : t.t0;
      const int64_t m = apply_transform(*t.P, code, cp, cn, dst, t.cap_t);
      if (m < 0) {
        t.flags |= GI_REQ_OVERFLOW;
        break;
      }
      changed = !((uint32_t)m == cn && eq_bytes(dst, (uint32_t)m, cp, cn));  // unchanged: no candidate
      if (changed) {
        cp = dst;
        cn = (uint32_t)m;
      }
    }
    fresh = changed;
  }
  return nm;
}

// Hit slot s is set only by per-value phase-A evaluation (each such hit also
// marks its value in the value map): not an always-slot.
GI_HD __forceinline__ bool slot_vexact(const DProgram& P, uint32_t s) {
  for (uint32_t k = 0; k < P.n_always; k++)
    if (P.always_slots[k] == s) return false;
  return true;
}

// Which value of field f a collection target vr of link R tests (side
// effect free): 0 none, 1 an exact phase-A match (the operator need not run
// again), 2 evaluate it.  Phase A tested every value of fields [0, nf_pa)
// this link reads: one whose value-map bit is clear set no hit bit at all,
// so it cannot match here (value-exact slots only: an always-slot is set
// without a value); with the exact hit set, a value with a set bit is
// decided by its key (exact key: a match; maybe key: evaluate; no key: no
// match).  *names: the key side is tested.
GI_HD __forceinline__ uint32_t field_filter(Tx& t, const DRule& R, const DVarRef& vr, uint32_t f, bool vskip,
                                                 bool vexact, bool* names) {
  const DProgram& P = *t.P;
  const Field fl = t.fields[f];
  if (!field_in(vr.var, fl.kind, names)) return 0;
  uint32_t hres = 2;
  if (vskip && f < t.nf_pa && fl.kind <= FK_FILE_SIZE) {  // phase-A item kinds only
    const uint32_t vb = 2 * f + (*names ? 1u : 0u);
    // a value a filter link's phase-A pattern rejects: only its capture record (3), or nothing
    const uint32_t out = ((R.flags2 & RF2_PA_FILTER) && t.crec) ? 3u : 0u;
    if (!((t.vmap[vb] >> ((uint32_t)R.hit_slot & 31u)) & 1u)) hres = out;
    else if (vexact) {
      hres = hset_lookup(t.hset, t.hmask, (uint32_t)R.hit_slot, vb);
      if (!hres) hres = out;
      else if (R.flags2 & RF2_PA_RELAXED) hres = 2;  // a superset automaton's hit: evaluate the value
    }
    if (!hres) return 0;
  }
  if (vr.key_mode == 1) {
    if (vr.ci ? !eq_ascii_ci(fl.k, fl.kn, P.strpool + vr.key_off, vr.key_len)
              : !eq_bytes(fl.k, fl.kn, P.strpool + vr.key_off, vr.key_len))
      return 0;
  } else if (vr.key_mode == 2) {
    if (!dfa_match(P, vr.key_dfa, fl.k, fl.kn, vr.ci != 0)) return 0;
  }
  if (vr.exc_count && key_excluded(t, vr, fl.k, fl.kn)) return 0;
  if (t.nrtgt && R.id != 0 && target_removed(t, R.id, vr.var, fl.k, fl.kn)) return 0;
  return hres;
}

// Rule.doEvaluate for one link -> number of matched values.  W: k_eval_wave
// (the request's whole wave runs the interpreter uniformly; collection
// fields are filtered 64 at a time).
template <bool W>
GI_HD __forceinline__ uint32_t eval_rule(Tx& t, const DRule& R) {
  const DProgram& P = *t.P;
  // a folded constant link (compile.cpp fold_program): the values of the TX
  // slots it reads are the same for every request that reaches it, so it
  // matches _pad2 values; only its per-match actions remain
  if (R.flags & RF_CONST) {
    for (uint32_t k = 0; k < R._pad2; k++) run_actions(t, R);
    return R._pad2;
  }
  // phase-A filter: a clear hit bit proves no value matches (exact); a set
  // bit (match or "maybe") falls through to the full evaluation below.
  if (R.hit_slot >= 0 && !t.pa_void && !bodydep_void(t, R)) {
    const uint32_t w = t.hits[(uint64_t)(R.hit_slot >> 5) * t.hstride];
    if (!((w >> (R.hit_slot & 31)) & 1u) && !((R.flags2 & RF2_PA_FILTER) && t.crec)) {
      // (a filter link with capture records on walks its values for their records: field_filter)
      if (!residual_live(t, R)) return 0;
      // phase A cleared every other target: only the residual (body-phase)
      // singles can match; test them without side effects, and evaluate the
      // whole link in order only if one does
      const DOp o = gi_cload(P.ops, (uint64_t)R.op);
      bool any = false;
      for (uint32_t vi = 0; vi < R.var_count && !any; vi++) {
        const DVarRef vr = gi_cload(P.vars, R.var_begin + vi);
        if (!vr.residual) continue;
        if (vr.var == S_REQUEST_BODY && t.body_spec && R.phase >= 2) continue;  // k_body's bit
        if (vr.var >= S_COUNT) {  // a body collection phase A never scans (multipart, XML): test its entries
          // (key filters ignored: a superset, the full evaluation below is
          // exact; multiMatch: any entry is a "maybe")
          uint32_t klo, khi, j = 0, je = t.nf;
          var_kinds(vr.var, &klo, &khi);
          if (t.kx) {
            j = klo <= khi ? t.kx[klo] : 0u;
            je = klo <= khi ? t.kx[khi + 1] : 0u;
          }
          for (; j < je && !any; j++) {
            const Field fl = t.fields[t.kx ? t.kx[12 + j] : j];
            bool names;
            if (!field_in(vr.var, fl.kind, &names)) continue;
            if (R.flags & RF_MULTIMATCH) {
              any = true;
              continue;
            }
            bool ok;
            const Str tv = transform(t, R, names ? fl.k : fl.v, names ? fl.kn : fl.vn, &ok);
            any = !ok || eval_op(t, o, tv.p, tv.n);
          }
          continue;
        }
        bool ok;
        uint8_t sb[24];
        const Str sv = single_val(t, vr.var, sb);
        const Str tv = transform(t, R, sv.p, sv.n, &ok);
        any = ok && eval_op(t, o, tv.p, tv.n);
      }
      if (!any) return 0;
    }
  }
  if (R.op < 0) {
    run_actions(t, R);
    return 1;
  }
  const DOp o = gi_cload(P.ops, (uint64_t)R.op);
  uint32_t nmatch = 0;
  // The link's targets as one sequence of candidate values, in Coraza's order
  // (variables in rule order; a collection's entries in field order, TX keys
  // static then created; a count target's count after its walk), tested at
  // ONE test_value site: test_value (chain, operator dispatch, capture,
  // matched-variable state, actions) is inlined once instead of once per kind
  // of target, which kept k_eval's code and register pressure several times
  // larger.
  uint8_t nbuf[24];        // a candidate formatted as a number (counts, integer TX values)
  uint32_t vi = 0;         // the variable being walked
  bool in_var = false;     // its walk has started
  DVarRef vr{};
  uint32_t j = 0, je = 0, cnt = 0, se = 0;  // walk position / end, count, TX: end of the static slots
  bool vskip = false, vexact = false;
  uint64_t wm = 0;         // k_eval_wave: survivors of the current 64-field block
  uint32_t wf = 0, wh = 0;
  bool wn = false;
  for (;;) {
    const uint8_t* cv = nullptr;
    const uint8_t* ck = nullptr;
    uint32_t cvn = 0, cvar = 0, ckn = 0;
    bool cex = false, conly = false, have = false;
    while (!have) {
      if (!in_var) {
        if (vi >= R.var_count) break;
        vr = gi_cload(P.vars, R.var_begin + vi);
        in_var = true;
        cnt = 0;
        j = je = 0;
        wm = 0;
        if (vr.var < S_COUNT) {  // a single: one candidate
          in_var = false;
          vi++;
          if (t.nrtgt && R.id != 0 && target_removed(t, R.id, vr.var, nullptr, 0)) continue;
          if (vr.count) {
            nbuf[0] = '1';
            cv = nbuf;
            cvn = 1;
          } else {
            const Str sv = single_val(t, vr.var, nbuf);
            cv = sv.p;
            cvn = sv.n;
          }
          cvar = vr.var;
          have = true;
          continue;
        }
        if (vr.var == V_TX) {
          // static slots: a literal key names at most one; a regex key the ones the
          // compiler listed (DProgram.txrx); no key all.  Then (no literal key) the
          // keys macro-key setvars created, in creation order.
          uint32_t sb = 0;
          se = P.n_slots;
          if (vr.key_mode == 1) {
            sb = vr.slot < 0 ? 0u : (uint32_t)vr.slot;
            se = vr.slot < 0 ? 0u : (uint32_t)vr.slot + 1;
          } else if (vr.key_mode == 2) {
            se = vr.key_len;
          }
          j = sb;
          je = se + ((vr.key_mode != 1 && t.dyn) ? ((const DynHdr*)t.dyn)->n : 0u);
          continue;
        }
        if (vr.var >= V_MATCHED_VAR) {  // the matched-variable state (t.mv is set: mv_used)
          MvState* m = t.mv;
          if (!m) {  // no state: only unreachable rules read it (compile.cpp fold_program)
            in_var = false;
            vi++;
            continue;
          }
          if (vr.var == V_MATCHED_VAR || vr.var == V_MATCHED_VAR_NAME) {
            in_var = false;
            vi++;
            if (vr.count) {
              nbuf[0] = '1';
              cv = nbuf;
              cvn = 1;
            } else if (vr.var == V_MATCHED_VAR) {
              cv = mv_curval(m);
              cvn = m->cur_vn;
            } else {
              cv = mv_curname(m);
              cvn = m->cur_nn;
            }
            cvar = vr.var;
            have = true;
            continue;
          }
          je = m->n;  // MATCHED_VARS(_NAMES): the entries as they stood when the link started
          continue;
        }
        // a collection: value-map / hit-set filtering (field_filter); multiMatch
        // links count candidates per value, so they always evaluate
        vskip = R.hit_slot >= 0 && !vr.count && !t.pa_void && !bodydep_void(t, R) &&
                slot_vexact(P, (uint32_t)R.hit_slot);
        vexact = vskip && t.hset && !(R.flags & RF_MULTIMATCH);
        uint32_t klo, khi;
        je = t.nf;
        var_kinds(vr.var, &klo, &khi);
        if (t.kx) {  // only the collection's own fields
          j = klo <= khi ? t.kx[klo] : 0u;
          je = klo <= khi ? t.kx[khi + 1] : 0u;
          if (vr.count && vr.key_mode == 0 && !vr.exc_count && !t.nrtgt) {  // &COLLECTION: the entry count
            cnt = je - j;
            j = je;
          }
        }
        continue;
      }
      // the walk of variable vi: its next candidate, if any
      if (vr.var == V_TX) {
        if (j < je) {
          const uint32_t si = j++;
          const uint8_t* nm;
          uint32_t nn;
          Slot sl;
          if (si < se) {
            const uint32_t sid = vr.key_mode == 2 ? P.txrx[vr.key_off + si] : si;
            sl = slot_rd(t, sid);
            if (sl.state == 0) continue;
            nm = P.strpool + P.slot_names[sid * 2];
            nn = P.slot_names[sid * 2 + 1];
          } else {
            const DynEnt& de = dyn_ents(t.dyn)[si - se];
            sl = de.s;
            if (sl.state == 0) continue;
            nm = de.k;
            nn = de.kn;
            if (vr.key_mode == 2) {
              if (vr.pre_len) {  // ^literal
                if (nn < vr.pre_len || !eq_bytes_w(nm, vr.pre_len, P.strpool + vr.slot, vr.pre_len)) continue;
              } else if (!dfa_match(P, vr.key_dfa, nm, nn, false)) {
                continue;
              }
            }
          }
          if (key_excluded(t, vr, nm, nn)) continue;
          if (t.nrtgt && R.id != 0 && target_removed(t, R.id, V_TX, nm, nn)) continue;
          if (vr.count) {
            cnt++;
            continue;
          }
          if (sl.state == 1 && R.tchain_len == 0 && o.has_num && o.kind >= OP_EQ && o.kind <= OP_LT) {
            // integer TX value against a numeric literal: eval_op would Atoi the
            // canonical decimal back to sl.num, so compare directly (an exact
            // candidate; its decimal only for the matched-variable state)
            const int64_t a = o.num, b = sl.num;
            bool res = o.kind == OP_EQ ? b == a : o.kind == OP_GE ? b >= a : o.kind == OP_GT ? b > a
                       : o.kind == OP_LE ? b <= a : b < a;
            if (o.negate) res = !res;
            if (!res) continue;
            cv = nbuf;
            cvn = t.mv ? go_itoa(sl.num, nbuf) : 0u;
            cex = true;
          } else {
            const Str sv = slot_str(t, sl, nbuf);
            cv = sv.p;
            cvn = sv.n;
          }
          cvar = V_TX;
          ck = nm;
          ckn = nn;
          have = true;
          continue;
        }
      } else if (vr.var >= V_MATCHED_VAR) {
        if (j < je) {
          const MvEnt e = mv_ents(t.mv)[j++];
          if (vr.key_mode == 1) {
            if (!eq_ascii_ci(e.name, e.nn, P.strpool + vr.key_off, vr.key_len)) continue;
          } else if (vr.key_mode == 2) {
            if (!dfa_match(P, vr.key_dfa, e.name, e.nn, true)) continue;
          }
          if (vr.exc_count && key_excluded(t, vr, e.name, e.nn)) continue;
          if (vr.count) {
            cnt++;
            continue;
          }
          const bool nms = vr.var == V_MATCHED_VARS_NAMES;
          cv = nms ? e.name : e.v;
          cvn = nms ? e.nn : e.vn;
          cvar = vr.var;
          ck = e.name;
          ckn = e.nn;
          have = true;
          continue;
        }
      } else {
        if constexpr (!W) {
          if (j < je) {
            const uint32_t f = t.kx ? t.kx[12 + j] : j;
            j++;
            bool names;
            const uint32_t hres = field_filter(t, R, vr, f, vskip, vexact, &names);
            if (!hres) continue;
            if (vr.count) {
              cnt++;
              continue;
            }
            const Field fl = t.fields[f];
            cv = names ? fl.k : fl.v;
            cvn = names ? fl.kn : fl.vn;
            cvar = vr.var;
            ck = fl.k;
            ckn = fl.kn;
            cex = hres == 1;
            conly = hres == 3;
            have = true;
            continue;
          }
        } else {
          // k_eval_wave: the lanes filter 64 fields at a time (pure: value map,
          // hit set, key selectors, exclusions), then the wave tests the
          // survivors in field order, uniformly (actions and matched-variable
          // state keep Coraza's per-value order)
          if (wm) {
            const int b = __ffsll((unsigned long long)wm) - 1;
            wm &= wm - 1;
            const uint32_t fb = (uint32_t)__shfl((int)wf, b, 64);
            const uint32_t hb = (uint32_t)__shfl((int)wh, b, 64);
            const bool nb = __shfl((int)wn, b, 64) != 0;
            const Field fl = t.fields[fb];
            cv = nb ? fl.k : fl.v;
            cvn = nb ? fl.kn : fl.vn;
            cvar = vr.var;
            ck = fl.k;
            ckn = fl.kn;
            cex = hb == 1;
            conly = hb == 3;
            have = true;
            continue;
          }
          if (j < je) {
            const uint32_t lane = threadIdx.x & 63u;
            const uint64_t c0 = t.profon ? gi_clock() : 0;
            wf = 0;
            wh = 0;
            wn = false;
            if (j + lane < je) {
              wf = t.kx ? t.kx[12 + j + lane] : j + lane;
              wh = field_filter(t, R, vr, wf, vskip, vexact, &wn);
            }
            const uint64_t m = __ballot(wh != 0);
            if (t.profon) {  // GI_PROF (lane 0): fields filtered, survivors exact / to evaluate, cycles
              unsigned long long* pf = t.prof_rule_cyc - 128;
              const uint64_t mx = __ballot(wh == 1);
              atomicAdd(&pf[17], (unsigned long long)min(64u, je - j));
              atomicAdd(&pf[18], (unsigned long long)__popcll(mx));
              atomicAdd(&pf[19], (unsigned long long)__popcll(m & ~mx));
              atomicAdd(&pf[20], (unsigned long long)(gi_clock() - c0));
            }
            j += 64;
            if (vr.count) cnt += (uint32_t)__popcll(m);
            else wm = m;
            continue;
          }
        }
      }
      // the walk of variable vi ended: a count target's candidate is its count
      in_var = false;
      vi++;
      if (vr.count) {
        cv = nbuf;
        cvn = go_itoa(cnt, nbuf);
        cvar = vr.var;
        have = true;
      }
    }
    if (!have) break;
    if (conly) {  // RF2_PA_FILTER: the value changes nothing but the capture records
      CapHdr* CH = (CapHdr*)t.capws;
      if (!CH->trunc) {
        // the link captures the whole t:lowercase value (compile.cpp within_chain_filters):
        // lowercase straight into the record row -- run_capture's record, without the call
        // or the TX.0 copy nobody reads (captures are not observable outside this chain).
        // One pass with no early exit (the loads pipeline): copy, then keep it if ASCII.
        const uint32_t nrec = CH->nrec, nbytes = CH->nbytes;
        bool ascii = cvn <= t.cap_t;
        bool fits = nrec < CH->rec_cap && nbytes + cvn <= CH->bytes_cap;
        if (ascii && fits) {
          uint8_t* d = CH->bytes + nbytes;
          uint32_t acc = 0;
          for (uint32_t i = 0; i < cvn; i++) {
            const uint8_t c = cv[i];
            acc |= c;
            d[i] = (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c;
          }
          ascii = acc < 0x80;
        } else if (ascii) {
          for (uint32_t i = 0; i < cvn && ascii; i++) ascii = cv[i] < 0x80;
        }
        if (ascii) {
          if (fits) {
            uint32_t* rr = CH->rec + 4ull * nrec;
            rr[0] = t.cur_id;
            rr[1] = 0u;
            rr[2] = nbytes;
            rr[3] = cvn;
            CH->nbytes = nbytes + cvn;
            CH->nrec = nrec + 1;
          } else {
            CH->trunc = 1;
          }
        } else {
          bool ok;
          const Str tv = transform(t, R, cv, cvn, &ok);
          if (ok) t.flags |= run_capture(*t.P, t.capws, t.capbuf, t.cap_t, t.slots, t.n_req, t.cur_id, o.pike, tv.p, tv.n);
        }
      }
      continue;
    }
    nmatch += test_value(t, R, o, cv, cvn, cvar, ck, ckn, cex);
  }
  return nmatch;
}

template <bool W>
GI_HD __forceinline__ void eval_top(Tx& t, uint32_t ri) {
  const DProgram& P = *t.P;
  const DRule R = gi_cload(P.rules, ri);
  // the rule and its chain links; all must match (one eval_rule call site)
  t.prof_evals++;
  t.cur_id = (uint32_t)R.id;
  t.cur_groups = P.n_rm_groups ? P.rule_groups[ri] : 0u;
  if (t.mv) {
    t.mv->keep = R.flags2 & RF2_MVS;
    t.mv->cur = R.flags2 & RF2_MVCUR;
  }
  for (int32_t ci = (int32_t)ri; ci >= 0;) {
    const DRule C = gi_cload(P.rules, (uint64_t)ci);
    const uint64_t c0 = t.profon ? gi_clock() : 0;
    const uint32_t o0 = t.prof_ops;
    const uint32_t nm = eval_rule<W>(t, C);
    if (t.profon) {
      const uint64_t dc = gi_clock() - c0;
      t.prof_eval_cyc += dc;
      if (ci < 1000) {  // cycles, lanes entering, operator runs (not phase-A exact) per link
        gi_prof_add(&t.prof_rule_cyc[ci], (unsigned long long)dc);
        gi_prof_add(&t.prof_rule_cyc[1000 + ci], 1ull);
        gi_prof_add(&t.prof_rule_cyc[2000 + ci], (unsigned long long)(t.prof_ops - o0));
      }
    }
    if (nm == 0) return;
    ci = C.chain_next;
  }
  t.prof_rules++;
  if (R.skip_after >= 0) t.skip_after = R.skip_after;
  if (R.skip) t.skip = R.skip;
  if ((R.disruptive == D_DENY || R.disruptive == D_DROP || R.disruptive == D_REDIRECT) && t.engine == ENGINE_ON) {
    t.interrupted = true;
    t.int_rule = R.id;
    t.int_status = R.status;
    t.int_action = R.disruptive == D_DENY ? GI_ACTION_DENY : R.disruptive == D_DROP ? GI_ACTION_DROP
                                                                                     : GI_ACTION_REDIRECT;
    t.int_phase = t.phase;
  } else if (R.disruptive >= D_ALLOW_ALL && t.engine == ENGINE_ON) {
    t.allow = R.disruptive;  // [upstream allow.go Evaluate: tx.AllowType]; eval_phase ends the walk
  }
  if (R.id != 0) {
    if (t.nmatched < t.mcap) t.mout[t.nmatched] = (uint32_t)R.id;
    else t.flags |= GI_REQ_MATCH_TRUNC;
    t.nmatched++;
  }
}

// Is rule index k of the phase walk a no-op for this request in the current
// state (no skip count pending)?  A removed rule, a marker we are not
// skipping to, a rule whose first link phase A cleared; with skipAfter
// pending, every rule but the target marker.  (Used by k_eval_wave to jump
// over runs of such rules 64 at a time; MATCHED_VARS is reset before every
// evaluated rule, so skipping the resets of no-op rules changes nothing.)
GI_HD __forceinline__ bool rule_noop(Tx& t, const DRule& R, uint32_t ri) {
  if (R.id != 0 && t.nremoved) {
    for (uint32_t j = 0; j < t.nremoved; j++)
      if (t.removed[j][0] <= R.id && R.id <= t.removed[j][1]) return true;
  }
  if (t.rm_groups && (t.P->rule_groups[ri] & t.rm_groups)) return true;
  if (t.skip_after >= 0) return R.marker != t.skip_after;
  if (R.flags & RF_MARKER) return true;
  if ((R.flags & RF_CONST) && R._pad2 == 0) return true;  // a folded link that matches nothing
  return R.hit_slot >= 0 && !residual_live(t, R) && !t.pa_void && !bodydep_void(t, R) &&
         !((t.hits[(uint64_t)(R.hit_slot >> 5) * t.hstride] >> (R.hit_slot & 31)) & 1u) &&
         !((R.flags2 & RF2_PA_FILTER) && t.crec);
}

// RuleGroup.Eval [upstream corazawaf/rulegroup.go]
template <bool W>
GI_HD __forceinline__ void eval_phase(Tx& t, uint8_t phase) {
  const DProgram& P = *t.P;
  if (t.engine == ENGINE_OFF) return;
  // an allow of an earlier phase: "allow" skips every later phase but logging,
  // "allow:request" the rest of the request phases -- both end here (phases 1, 2)
  if (t.allow == D_ALLOW_ALL || t.allow == D_ALLOW_REQUEST) return;
  t.phase = phase;
  const uint32_t kend = P.top_end[phase - 1];
  const uint32_t k0 = P.top_begin[phase - 1];
  if (phase == 1 && P.fold_on) {
    // the folded request-independent rules (compile.cpp fold_program): their
    // TX effects are the snapshot from here on (ids: where the walk reaches them)
    t.snap = true;
    for (uint32_t s = 128; s < P.n_slots; s++) TXS(t, s) = ((const Slot*)P.tx_snap)[s];
    if (t.capws)
      for (uint32_t g = 0; g < 9; g++)
        if (P.cap_slots[g] >= 0) TXS(t, P.cap_slots[g]) = ((const Slot*)P.tx_snap)[P.cap_slots[g]];
  }
  for (uint32_t k = k0; k < kend; k++) {
    if (t.interrupted) break;
    if (t.flags & GI_REQ_ERROR_MASK) break;
    if constexpr (W) {
      if (t.skip == 0) {
        // the lanes test the next 64 rules; jump to the first that is not a no-op
        const uint32_t kk = k + (threadIdx.x & 63u);
        bool need = false;
        if (kk < kend) {
          const uint32_t rl = GI_CONST(uint32_t, P.top)[kk];
          const DRule Rl = P.rules[rl];
          need = !rule_noop(t, Rl, rl);
        }
        const uint64_t m = __ballot(need);
        if (!m) {
          k += 63;
          continue;
        }
        k += (uint32_t)(__ffsll((unsigned long long)m) - 1);
      }
    }
    const uint32_t ri = GI_CONST(uint32_t, P.top)[k];
    const DRule R = gi_cload(P.rules, ri);
    t.prof_visits++;
    const int32_t id = R.id;
    if (id != 0 && t.nremoved) {
      bool rm = false;
      for (uint32_t j = 0; j < t.nremoved; j++)
        if (t.removed[j][0] <= id && id <= t.removed[j][1]) rm = true;
      if (rm) continue;
    }
    if (t.rm_groups && (P.rule_groups[ri] & t.rm_groups)) continue;  // ctl:ruleRemoveByTag / ByMsg
    if (t.skip_after >= 0) {
      if (R.marker == t.skip_after) t.skip_after = -1;
      continue;
    }
    if (t.skip > 0) {
      t.skip--;
      continue;
    }
    if (R.flags & RF_MARKER) continue;
    if (R.flags & RF_FOLDED) {
      // a run of folded rules (compile.cpp fold_program): their TX effects are
      // the snapshot, their matched ids are fixed; the walk continues after it
      const uint32_t* fr = P.fold_runs + 4ull * R._pad2;
      for (uint32_t i = 0; i < fr[1]; i++) {
        if (t.nmatched < t.mcap) t.mout[t.nmatched] = P.fold_ids[fr[0] + i];
        else t.flags |= GI_REQ_MATCH_TRUNC;
        t.nmatched++;
      }
      t.skip_after = (int32_t)fr[3];
      k = fr[2] - 1;
      continue;
    }
    if (t.mv) {  // RuleGroup.Eval resets MATCHED_VARS(_NAMES) before each rule
      t.mv->n = 0;
      t.mv->nb = 0;
    }
    if (R.hit_slot >= 0 && !residual_live(t, R) && !t.pa_void && !bodydep_void(t, R) &&
        !((t.hits[(uint64_t)(R.hit_slot >> 5) * t.hstride] >> (R.hit_slot & 31)) & 1u) &&
        !((R.flags2 & RF2_PA_FILTER) && t.crec))
      continue;  // phase A proved the first link matches nothing (a filter link: and records no capture)
    if ((R.flags & RF_CONST) && R._pad2 == 0) continue;  // folded: matches nothing for any request
    if (t.prefix && (R.flags2 & RF2_BODY_PA)) {  // needs the body's phase-A scan: the first stage ends here
      t.bail = true;
      break;
    }
    eval_top<W>(t, ri);
    if (t.allow) {  // the allow rule ends this phase's walk (allow:phase: only this one)
      if (t.allow == D_ALLOW_PHASE) t.allow = 0;
      break;
    }
    // a skipAfter the rule just set: the rules up to its marker are all
    // skipped (no side effects), so resume at the marker entry directly
    if (t.skip_after >= 0) k = GI_CONST(uint32_t, P.top_jump)[k] - 1;
  }
}

// ------------------------------------------------------ per-request state
// Written by k_collect at the start of the request's HBM scratch region and
// read by k_match / k_eval.
struct ReqHdr {
  uint32_t nf;          // fields so far: [ARG_GET | HEADER | COOKIE | ARG_POST]
  uint32_t nb;          // bytes arena used
  uint16_t n_get, n_hdr, n_ck, flags;
  uint8_t body_proc;
  uint8_t pa_void;      // phase-A arena overflowed: k_eval ignores the hit bits
  uint8_t spec_proc;    // body processor k_bparse parsed the body with (BP_NONE: none)
  uint8_t spec_err;     // its body-error class (multipart MpErr; 0 none)
  uint32_t n_post;      // its fields (ARGS_POST, multipart collections), after the phase-1 fields
  Str single[S_COUNT];
};
static_assert(sizeof(ReqHdr) <= GI_REQHDR_BYTES, "ReqHdr must fit its slot");

struct Region {
  ReqHdr* hdr;
  Field* fields;
  Slot* slots;
  uint8_t *bytes, *t0, *t1, *mt, *txa;
  int64_t (*rm)[2];
  uint32_t* capws;
  uint8_t* capbuf;
  MvState* mv;
  uint8_t* dyn;  // dynamic TX area (DynHdr), nullptr when the program has no macro-key setvar
  uint32_t cap_f, cap_b, cap_t, cap_mt;
};

GI_HD inline Region region_of(const DProgram& P, const DBatch& B, uint32_t r) {
  const ReqLayout L = B.layout[r];
  uint8_t* base = B.scratch + L.base;
  Region g;
  g.hdr = (ReqHdr*)base;
  uint64_t off = GI_REQHDR_BYTES;
  g.fields = (Field*)(base + off);
  off += (uint64_t)L.cap_f * sizeof(Field);
  g.slots = (Slot*)(base + off);
  off += ((uint64_t)P.n_slots * sizeof(Slot) + 15) & ~15ull;
  g.rm = (int64_t(*)[2])(base + off);
  off += GI_RM_BYTES;
  g.bytes = base + off;
  off += (L.cap_b + 15) & ~15u;
  g.t0 = base + off;
  off += (L.cap_t + 15) & ~15u;
  g.t1 = base + off;
  off += (L.cap_t + 15) & ~15u;
  g.mt = base + off;
  off += (L.cap_mt + 15) & ~15u;
  g.txa = base + off;
  off += (L.cap_mt + 15) & ~15u;
  g.dyn = P.n_dyn_sites ? base + off : nullptr;
  off += P.n_dyn_sites ? 16ull + 32ull * L.dyn_cap + L.dyn_capb : 0ull;
  // observable captures: the submatch workspace and one value buffer per group,
  // in the chunk's capture pool (runtime.cpp sizes a chunk to fit it)
  g.capws = P.cap_ws_words ? (uint32_t*)(B.cappool + L.cap_off) : nullptr;
  g.capbuf = P.cap_ws_words ? B.cappool + L.cap_off + (((uint64_t)P.cap_ws_words * 4 + 15) & ~15ull) : nullptr;
  g.mv = P.mv_used ? (MvState*)(base + off) : nullptr;
  g.cap_f = L.cap_f;
  g.cap_b = L.cap_b;
  g.cap_t = L.cap_t;
  g.cap_mt = L.cap_mt;
  return g;
}

GI_HD inline void tx_bind(Tx& t, const DProgram& P, const Region& g) {
  t.P = &P;
  t.fields = g.fields;
  t.cap_f = g.cap_f;
  t.slots = g.slots;
  t.bytes = g.bytes;
  t.cap_b = g.cap_b;
  t.t0 = g.t0;
  t.t1 = g.t1;
  t.cap_t = g.cap_t;
  t.mt = g.mt;
  t.cap_mt = g.cap_mt;
  t.txa = g.txa;
  t.removed = g.rm;
  t.rtgt = (Tx::RmTarget*)(g.rm + 8);
  t.cap_tx = g.cap_mt;
  t.single = g.hdr->single;
  t.mv = g.mv;
  t.capws = g.capws;
  t.capbuf = g.capbuf;
  t.dyn = g.dyn;
}

GI_HD inline bool validate_op(uint8_t kind, const uint32_t* bits, const uint8_t* s, uint32_t n) {
  if (kind == OP_UNCONDITIONAL) return true;  // a count link's "an admitted entry exists" (compile.cpp plan)
  if (kind == OP_VALIDATE_BYTE_RANGE) {
    for (uint32_t i = 0; i < n; i++)
      if (!((bits[s[i] >> 5] >> (s[i] & 31)) & 1)) return true;
    return false;
  }
  if (kind == OP_VALIDATE_URL_ENCODING) {
    for (uint32_t i = 0; i < n;) {
      if (s[i] == '%') {
        if (i + 2 >= n) return true;
        if (ishex(s[i + 1]) && ishex(s[i + 2])) i += 3;
        else return true;
      } else {
        i++;
      }
    }
    return false;
  }
  for (uint32_t i = 0; i < n;) {  // OP_VALIDATE_UTF8
    uint32_t w;
    uint32_t r = decode_rune(s, n, i, &w);
    if (r == 0xFFFD && w == 1) return true;
    i += w;
  }
  return false;
}

// Debug builds (-DGI_DEBUG): bounds violations are recorded in B.dbg
// ([0] first source line, [1] count, [2..3] operands) and the access skipped.
#ifdef GI_DEBUG
GI_HD __noinline__ void gi_dbg_fail(const DBatch& B, uint32_t line, uint64_t a, uint64_t b) {
  if (!B.dbg) return;
  if (atomicCAS(&B.dbg[0], 0u, line) == 0u) {
    B.dbg[2] = (uint32_t)a;
    B.dbg[3] = (uint32_t)b;
  }
  atomicAdd(&B.dbg[1], 1u);
}
#define GI_BOUND(cond, a, b)                        \
  do {                                              \
    if (!(cond)) {                                  \
      gi_dbg_fail(B, __LINE__, (a), (b));           \
      return;                                       \
    }                                               \
  } while (0)
#else
#define GI_BOUND(cond, a, b) \
  do {                       \
  } while (0)
#endif

__device__ inline void set_hit(const DBatch& B, uint32_t slot, uint32_t r) {
  GI_BOUND(r < B.n_req && slot < B.n_hit_slots, slot, r);
  atomicOr(&B.hits[(uint64_t)(slot >> 5) * B.rstride + r], 1u << (slot & 31));
}

// cause (GI_VOID_*): which capacity ran out (counted in B.vcause for GI_DIAG)
#define GI_VOID_FIELD 0
#define GI_VOID_LONG 1
#define GI_VOID_SLOW 2
#define GI_VOID_QCAP 3
#define GI_VOID_POOL 4
#define GI_VOID_DEDUP 5  // a header copy whose canonical occurrence's results are not exactly known
GI_HD __forceinline__ void void_request(const DBatch& B, uint32_t r, uint32_t cause) {
  ReqHdr* H = (ReqHdr*)(B.scratch + B.layout[r].base);
  H->pa_void = 1;
  atomicAdd(&B.vcause[cause], 1ull);
}

#define GI_NB 5  // item length buckets: <=16, <=32, <=64, <=128, >128 bytes
// qblk entry {pool word offset, nv | nw << 8 | shared}: shared = the block was
// written for an earlier stream of the same item-wave (raw item bytes)
#define GI_QB_SHARED 0x80000000u
#define GI_QB_BODY 0x40000000u  // every value of the block is a body field (the gate: DJob.prefix selects the jobs)
#define GI_QB_HDR 2  // lane header words of a queue block: global item index, value length
#define GI_QB_NW_MASK 0x3FFFFFu
// The gate (launch_pipeline): does this stage run a job / value test (its
// DJob.prefix / DScanVal.prefix) over a body field (body) or a phase-1 item?
// The first stage runs every one over phase-1 items and the prefix ones over
// body fields; the body stage (body fields only) the others.
__device__ __forceinline__ bool stage_runs(const DBatch& B, bool body, uint8_t prefix) {
  return B.stage == 0 || (B.stage == 1 ? (!body || prefix) : (body && !prefix));
}
GI_HD __forceinline__ uint32_t item_bucket(uint32_t n) {
  return n <= 16 ? 0u : n <= 32 ? 1u : n <= 64 ? 2u : n <= 128 ? 3u : 4u;
}
// Item classes: k_items orders the items of each bucket by (source group,
// length class), so the 64 values of an item wave come from one kind of
// variable (singles; ARGS_GET / ARGS_POST / headers / cookies / FILES*
// values or keys) and have (nearly) one length.  The streams that do not
// admit that kind are then skipped by the whole wave (k_stream), and the
// lanes of a chain or of k_scan's lockstep automata run out of work together.
// Length classes per bucket: one per length up to 128 bytes, then 16 ranges
// of 128 bytes (the last open); bucket b holds 16 groups x kNl[b] classes.
__constant__ uint32_t kClsLo[GI_NB] = {0, 17, 33, 65, 129};
__constant__ uint32_t kClsN[GI_NB] = {17, 16, 32, 64, 16};
__constant__ uint32_t kClsBase[GI_NB + 1] = {0, 272, 528, 1040, 2064, 2320};
__device__ __forceinline__ uint32_t item_class(uint32_t kind, uint32_t side, uint32_t n) {
  const uint32_t b = item_bucket(n);
  const uint32_t g = kind ? ((kind << 1) | side) & 15u : 0u;
  const uint32_t lc = b < 4 ? n - kClsLo[b] : min(15u, (n - 129u) / 128u);
  return kClsBase[b] + g * kClsN[b] + lc;
}

// one source group's classes, numbered 0 .. GI_NCLS / 16 - 1 (k_bparse's
// per-body counts of the ARGS_POST groups), and back to the global class
__device__ __forceinline__ uint32_t item_class_in_group(uint32_t n) {
  const uint32_t b = item_bucket(n);
  const uint32_t lc = b < 4 ? n - kClsLo[b] : min(15u, (n - 129u) / 128u);
  uint32_t pre = 0;
  for (uint32_t k = 0; k < b; k++) pre += kClsN[k];
  return pre + lc;
}
__device__ __forceinline__ uint32_t item_class_of_group(uint32_t g, uint32_t r) {
  uint32_t b = 0;
  while (b + 1 < GI_NB && r >= kClsN[b]) {
    r -= kClsN[b];
    b++;
  }
  return kClsBase[b] + g * kClsN[b] + r;
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// rank of this lane among the lanes of mask below it
__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t x, uint32_t* total) {
  const uint32_t L = lane_id();
  uint32_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (L >= (uint32_t)o) inc += y;
  }
  *total = __shfl(inc, 63, 64);
  return inc - x;
}

GI_HD __forceinline__ uint32_t wave_max(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o, 64));
  return x;
}

// Sum over the wave's 64 lanes (every lane gets it).
GI_HD __forceinline__ uint64_t wave_sum(uint64_t x) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, o, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), o, 64);
    x += ((uint64_t)hi << 32) | lo;
  }
  return x;
}

// Visits the items of one request: singles some filter reads, then the
// (value, key) sides of every field kind some filter reads.  part (the gate,
// launch_pipeline): 0 all items, 1 the phase-1 items (no body field), 2 the
// body fields alone.
template <class F>
GI_HD __forceinline__ void for_each_item(const DProgram& P, const ReqHdr* H, const Field* Fd, F&& f,
                                         uint32_t part = 0, bool dedup = false) {
  if (part != 2)
    for (uint32_t m = P.item_singles; m; m &= m - 1) {
      const uint32_t sg = __ffs(m) - 1;
      f((uint8_t)0, (uint8_t)sg, 0u, (uint32_t)0xFFFFFFFFu, H->single[sg].n);
    }
  const uint32_t n_get = H->n_get, n_hdr = H->n_hdr, n_ck = H->n_ck, n_pre = n_get + n_hdr + n_ck;
  const uint32_t i_end = part == 1 ? n_pre : n_pre + H->n_post;
  for (uint32_t i = part == 2 ? n_pre : 0u; i < i_end; i++) {
    const Field fl = Fd[i];
    // the body range may hold multipart collections: FILES / FILES_NAMES /
    // FILES_SIZES are phase-A items, part headers are not
    const uint8_t kind = i < n_get ? FK_ARG_GET : i < n_get + n_hdr ? FK_HEADER : i < n_pre ? FK_COOKIE : (uint8_t)fl.kind;
    if (kind < FK_ARG_GET || kind > FK_FILE_SIZE) continue;
    // (a header side k_collect found a copy of elsewhere in the chunk: no item,
    // k_dspread copies the copy's phase-A results -- Field._pad bit = side)
    const uint8_t sides = P.item_sides[kind] & (dedup && kind == FK_HEADER ? ~(uint8_t)fl._pad : 0xFFu);
    if (sides & 1) f(kind, (uint8_t)0, 0u, i, fl.vn);
    if (sides & 2) f(kind, (uint8_t)0, 1u, i, fl.kn);
  }
}

// ------------------------------------------------ stage 1: k_collect
// ProcessURI + AddRequestHeader* for one request per thread.  Fields are
// grouped by kind so each scan group walks only its own range.
GI_HD void collect_request(const DProgram& P, const DBatch& B, uint32_t r) {
  const gi_request rq = B.reqs[r];
  Region g = region_of(P, B, r);
  Tx t;
  tx_bind(t, P, g);
  t.nf = 0;
  t.nb = 0;
  t.flags = 0;
  t.body_proc = BP_NONE;
  for (uint32_t s = 0; s < S_COUNT; s++) t.single[s] = {CS_ZERO, 0};
  t.single[S_REQBODY_ERROR] = {CS_ZERO, 1};
  t.single[S_MULTIPART_STRICT_ERROR] = {CS_ZERO, 1};
  const uint8_t* D = B.data;
  Str method{D + rq.method.off, rq.method.len};
  Str uri{D + rq.uri.off, rq.uri.len};
  Str proto{D + rq.proto.off, rq.proto.len};
  t.single[S_REQUEST_METHOD] = method;
  t.single[S_REQUEST_PROTOCOL] = proto;
  t.single[S_REMOTE_ADDR] = {D + rq.remote_addr.off, rq.remote_addr.len};
  t.single[S_SERVER_NAME] = {D + rq.server_name.off, rq.server_name.len};
  {  // REMOTE_PORT: strconv.Itoa(port)
    uint8_t* pb = tx_alloc(t, 12);
    if (pb) {
      const uint32_t pn = go_itoa((int64_t)rq.remote_port, pb);
      t.nb -= 12 - pn;
      t.single[S_REMOTE_PORT] = {pb, pn};
    }
  }
  uint8_t* ln = tx_alloc(t, method.n + uri.n + proto.n + 2);
  if (ln) {
    uint32_t k = 0;
    copy_bytes(ln + k, method.p, method.n);
    k += method.n;
    ln[k++] = ' ';
    copy_bytes(ln + k, uri.p, uri.n);
    k += uri.n;
    ln[k++] = ' ';
    copy_bytes(ln + k, proto.p, proto.n);
    k += proto.n;
    t.single[S_REQUEST_LINE] = {ln, k};
  }
  const bool ok = process_uri(t, uri.p, uri.n);
  const uint32_t n_get = t.nf;
  // SecArgumentsLimit [upstream transaction.go AddGetRequestArgument / checkArgumentLimit]:
  // an argument is dropped once ARGS_GET holds `limit` distinct keys -- which ones
  // depends on Go's map order (urlutil.ParseQuery), so a request that can reach
  // the limit (more than `limit` arguments) is flagged instead of guessed
  if (n_get > P.args_limit) t.flags |= GI_REQ_UNSUPPORTED_URI;
  if (ok) {
    for (uint32_t h = 0; h < rq.hdr_count; h++) {
      const gi_header hd = B.headers[rq.hdr_begin + h];
      if (hd.name.len == 0) continue;
      const uint8_t* k = D + hd.name.off;
      const uint8_t* v = D + hd.value.off;
      add_field(t, FK_HEADER, k, hd.name.len, v, hd.value.len);
      if (hd.name.len == 12 && starts_ci(k, 12, "content-type")) {
        if (starts_ci(v, hd.value.len, "application/x-www-form-urlencoded")) {
          t.body_proc = BP_URLENCODED;
          t.single[S_REQBODY_PROCESSOR] = {CS_URLENCODED, 10};
        } else if (starts_ci(v, hd.value.len, "multipart/form-data")) {
          t.body_proc = BP_MULTIPART;
          t.single[S_REQBODY_PROCESSOR] = {CS_MULTIPART, 9};
        }
      }
    }
  }
  const uint32_t n_hdr = t.nf - n_get;
  if (ok) {
    for (uint32_t h = 0; h < rq.hdr_count; h++) {
      const gi_header hd = B.headers[rq.hdr_begin + h];
      if (hd.name.len == 6 && starts_ci(D + hd.name.off, 6, "cookie"))
        parse_cookies(t, D + hd.value.off, hd.value.len);
    }
  }
  ReqHdr* H = g.hdr;
  H->nf = t.nf;
  H->n_get = (uint16_t)n_get;
  H->n_hdr = (uint16_t)n_hdr;
  H->n_ck = (uint16_t)(t.nf - n_get - n_hdr);
  H->flags = t.flags | ((t.nf > 0xFFFF) ? GI_REQ_OVERFLOW : 0);
  H->body_proc = t.body_proc;
  H->pa_void = 0;
  // Speculative ProcessRequestBody so phase A also scans ARGS_POST: the
  // processor Content-Type implies (Coraza's own URLENCODED default, or JSON
  // for a "json" media type as the CRS ctl:requestBodyProcessor rules pick
  // it).  The fields sit after the phase-1 fields; k_eval uses them (and
  // trusts the hit bits of links that read ARGS_POST) only if phase 1 ends
  // with the same processor, and parses the body itself otherwise.
  uint8_t sp = BP_NONE;
  const uint32_t bn = rq.body.len;
  if (ok && P.body_access && bn > 0 && bn <= P.body_limit && !(t.flags & GI_REQ_ERROR_MASK)) {
    sp = t.body_proc;
    if (sp == BP_NONE) {
      for (uint32_t h = 0; h < rq.hdr_count && sp == BP_NONE; h++) {
        const gi_header hd = B.headers[rq.hdr_begin + h];
        if (hd.name.len == 12 && starts_ci(D + hd.name.off, 12, "content-type") &&
            contains_ci(D + hd.value.off, hd.value.len, "json"))
          sp = BP_JSON;
      }
    }
    if (sp != BP_URLENCODED && sp != BP_JSON && sp != BP_MULTIPART) sp = BP_NONE;
  }
  H->spec_proc = sp;  // k_bparse parses the body (or resets this to BP_NONE)
  H->spec_err = 0;
  H->n_post = 0;
  H->nb = t.nb;
}

// The first Content-Type request header's value (coraza ProcessRequestBody's mime)
GI_HD inline Str first_content_type(const DBatch& B, const gi_request& rq) {
  for (uint32_t h = 0; h < rq.hdr_count; h++) {
    const gi_header hd = B.headers[rq.hdr_begin + h];
    if (hd.name.len == 12 && eq_ascii_ci(B.data + hd.name.off, 12, (const uint8_t*)"content-type", 12))
      return {B.data + hd.value.off, hd.value.len};
  }
  return {CS_ZERO, 0};
}

GI_HD inline Str mp_err_msg(uint8_t e) {
  const uint8_t* m = (const uint8_t*)kMpErrMsg[e];
  uint32_t k = 0;
  while (m[k]) k++;
  return {m, k};
}

// Speculative ProcessRequestBody (k_collect picked the processor): one wave
// per body.  urlencoded bodies are split over the lanes: a field is a
// non-empty '&'-separated segment, so lane L takes the segments that start in
// its 1/64 of the body (a wave prefix sum numbers them in body order) and
// decodes each key / value into the arena at the segment's own offset (a
// decoding is never longer than its input, so segments cannot collide).  JSON
// bodies run the sequential parser on lane 0.  A body that does not parse as
// guessed (or overflows a capacity) leaves no fields: k_eval decides.  The
// wave then adds the body fields' phase-A item counts to its k_collect
// block's bucket counts.
__device__ __forceinline__ void urlenc_segment(const uint8_t* q, uint32_t n, uint32_t p, uint32_t* j_out,
                                               uint32_t* e_out, bool* kesc, bool* vesc) {
  uint32_t j = p, e = 0xFFFFFFFFu;
  bool ke = false, ve = false;
  for (; j < n; j++) {
    const uint8_t c = q[j];
    if (c == '&') break;
    if (c == '=' && e == 0xFFFFFFFFu) e = j;
    else if (c == '%' || c == '+') (e == 0xFFFFFFFFu ? ke : ve) = true;
  }
  *j_out = j;
  *e_out = e == 0xFFFFFFFFu ? j : e;
  *kesc = ke;
  *vesc = ve;
}

// ---------------------------------------------------- wave-uniform JSON parse
// parse_json_body restated for one wave: every lane runs the same control
// flow on the same (uniform) parser state, so the wave can do the byte work
// 64 bytes at a time -- a string's end is one ballot over 64 bytes of an LDS
// window of the body, a flattened key is built in an LDS path buffer (a
// member's key extends its container's, which is a prefix of it) and copied
// to the arena by the lanes together, and its hash is a wave reduction.  The
// fields, their order, the arena allocations and the limits are exactly
// parse_json_body's; whatever it would reject (syntax, limits, capacity) or
// this restatement cannot hold (a key longer than the path buffer) returns
// false: the speculative parse then leaves no fields and k_eval parses the
// body itself.  Repeated keys: a parallel insert into a hash table of the key
// hashes finds whether any key repeats; if one does, lane 0 runs the
// sequential json_fold_keys (the fold itself is rare).
#define GI_JW_PATH 1024
struct JWFrame {
  uint32_t koff, kn;  // the container's own key (offset into the arena)
  uint32_t count;
  uint32_t is_arr;
  uint32_t h;         // its hash (wave_key_hash)
};

// decimal digits of v, and the digits written to d[0, nd)
__device__ __forceinline__ uint32_t dec_len(uint32_t v) {
  uint32_t nd = 1;
  for (; v >= 10; v /= 10) nd++;
  return nd;
}
template <class D>
__device__ __forceinline__ void dec_put(uint32_t v, uint32_t nd, D* d) {
  for (uint32_t k = nd; k > 0; k--) {
    d[k - 1] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
}

// LDS written by some lanes of the (single-wave) workgroup, read by others:
// LDS operations of one wave execute in order, so only the compiler must not
// move them across this point -- unlike __syncthreads, no wait for the
// wave's outstanding global stores (the parser's field and key stores)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct JWin {  // q[wb, we) is in win
  const uint8_t* q;
  gi_lds_u8* win;
  uint32_t n, W, wb, we;
  uint64_t rc;  // GI_PROF: cycles in refills
  uint32_t nr;  // refills
};

__device__ __forceinline__ void jw_refill(JWin& w, uint32_t i) {
  const uint64_t c0 = gi_clock();
  w.nr++;
  wave_lds_sync();  // every lane is done reading the old window
  w.wb = i & ~3u;
  w.we = min(w.n, w.wb + w.W);
  for (uint32_t k = w.wb + lane_id(); k < w.we; k += 64) w.win[k - w.wb] = w.q[k];
  wave_lds_sync();
  w.rc += gi_clock() - c0;
}
// byte i (i < n) of the body; the window moves forward (or back) to cover it
__device__ __forceinline__ uint8_t jw_at(JWin& w, uint32_t i) {
  if (i < w.wb || i >= w.we) jw_refill(w, i);
  return w.win[i - w.wb];
}
// the window covers [i, min(i + k, n)) (k <= W - 4)
__device__ __forceinline__ void jw_cover(JWin& w, uint32_t i, uint32_t k) {
  if (i < w.wb || min(i + k, w.n) > w.we) jw_refill(w, i);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, 64);
  return x;
}

// a hash of a key: the wave sum of jw_hmix(byte j, j) over its bytes (the
// lane holding byte j mixes it), ^ its length -- equal keys hash equal; the
// slow and the fast member paths compute the same function
__device__ __forceinline__ uint32_t jw_hmix(uint32_t b, uint32_t j) {
  uint32_t x = (b | (j << 8)) * 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  return x;
}
__device__ __forceinline__ uint32_t wave_key_hash(const gi_lds_u8* path, uint32_t kn) {
  uint32_t acc = 0;
  for (uint32_t j = lane_id(); j < kn; j += 64) acc += jw_hmix(path[j], j);
  return wave_sum(acc) ^ (kn * 0x27D4EB2Fu);
}

// json_string_end over the window: the string whose quote is at i
__device__ uint32_t jw_string_end(JWin& w, uint32_t i, bool* esc) {
  const uint32_t L = lane_id();
  *esc = false;
  uint32_t p = i + 1;
  while (true) {
    if (p >= w.n) return 0;
    jw_cover(w, p, 64);
    const uint32_t x = p + L;
    const uint8_t c = x < w.we ? w.win[x - w.wb] : (uint8_t)'a';
    const uint64_t m = __ballot(x < w.n && (c == '"' || c == '\\' || c < 0x20));
    if (!m) {
      p += 64;
      continue;
    }
    p += (uint32_t)(__ffsll((unsigned long long)m) - 1);
    const uint8_t c0 = w.win[p - w.wb];
    if (c0 == '"') return p + 1;
    if (c0 < 0x20) return 0;
    if (p + 1 >= w.n) return 0;
    const uint8_t e = jw_at(w, p + 1);
    *esc = true;
    if (e == 'u') {
      if (p + 6 > w.n) return 0;
      for (uint32_t k = 2; k < 6; k++)
        if (!ishex(jw_at(w, p + k))) return 0;
      p += 6;
      continue;
    }
    if (e != '"' && e != '\\' && e != '/' && e != 'b' && e != 'f' && e != 'n' && e != 'r' && e != 't') return 0;
    p += 2;
  }
}

// json_unescape of the validated string body q[i, i + n) into d (global or
// LDS); lane 0 stores when `one`
template <class D>
__device__ uint32_t jw_unescape(JWin& w, uint32_t i, uint32_t n, D* d, bool one) {
  const bool st = !one || lane_id() == 0;
  uint32_t o = 0, k = 0;
  uint8_t u[4];
  while (k < n) {
    const uint8_t c = jw_at(w, i + k);
    if (c != '\\') {
      if (st) d[o] = c;
      o++;
      k++;
      continue;
    }
    const uint8_t e = jw_at(w, i + k + 1);
    if (e != 'u') {
      if (st) d[o] = e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e;
      o++;
      k += 2;
      continue;
    }
    uint32_t r = 0;
    for (uint32_t b = 0; b < 4; b++) r = (r << 4) | hexv(jw_at(w, i + k + 2 + b));
    k += 6;
    if (r >= 0xD800 && r < 0xE000) {  // utf16.IsSurrogate: consume a following \uXXXX
      if (n - k >= 6 && jw_at(w, i + k) == '\\' && jw_at(w, i + k + 1) == 'u') {
        uint32_t r2 = 0;
        for (uint32_t b = 0; b < 4; b++) r2 = (r2 << 4) | hexv(jw_at(w, i + k + 2 + b));
        k += 6;
        r = (r < 0xDC00 && r2 >= 0xDC00 && r2 < 0xE000) ? 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00) : 0xFFFD;
      } else {
        r = 0xFFFD;
      }
    }
    const uint32_t un = utf8_put(r, u);
    if (st)
      for (uint32_t b = 0; b < un; b++) d[o + b] = u[b];
    o += un;
  }
  return o;
}

__device__ uint32_t jw_number_end(JWin& w, uint32_t i) {
  const uint32_t n = w.n;
  auto dg = [&](uint32_t k) { const uint8_t c = jw_at(w, k); return c >= '0' && c <= '9'; };
  if (i < n && jw_at(w, i) == '-') i++;
  if (i >= n || !dg(i)) return 0;
  if (jw_at(w, i) == '0') {
    i++;
  } else {
    while (i < n && dg(i)) i++;
  }
  if (i < n && jw_at(w, i) == '.') {
    i++;
    if (i >= n || !dg(i)) return 0;
    while (i < n && dg(i)) i++;
  }
  if (i < n && (jw_at(w, i) == 'e' || jw_at(w, i) == 'E')) {
    i++;
    if (i < n && (jw_at(w, i) == '+' || jw_at(w, i) == '-')) i++;
    if (i >= n || !dg(i)) return 0;
    while (i < n && dg(i)) i++;
  }
  return i;
}

// bits [a, 64) / [a, b) of a 64-bit mask
__device__ __forceinline__ uint64_t jw_from(uint32_t a) { return a >= 64 ? 0ull : ~0ull << a; }
__device__ __forceinline__ uint64_t jw_range(uint32_t a, uint32_t b) { return jw_from(a) & ~jw_from(b); }
__device__ __forceinline__ bool jw_bit(uint64_t m, uint32_t p) { return p < 64 && ((m >> p) & 1ull); }

// wave_parse_json's member step from 64 bytes of the window at i, lane L
// holding byte i + L, every test a ballot mask: a container's close, or
// [','] '"' name '"' ':' value / [','] value with the value a container
// opener, an unescaped string, a number or a literal -- all inside the 64
// bytes.  Its state changes (fields, arena, key path, frames, i, d) are the
// ones the general path makes for that member, in the same order; anything
// else returns 0 before changing anything (the general path then runs).
__device__ int jw_fast_member(const Region& g, JWin& w, const uint8_t* q, uint32_t& i, uint32_t& d, uint32_t& nf,
                              uint32_t& nb, uint64_t& jb, uint64_t lim, gi_lds_u8* path, JWFrame* st) {
  const uint32_t L = lane_id();
  const uint32_t n = w.n;
  if (i >= n) return 0;
  jw_cover(w, i, 64);
  const uint32_t cl = min(64u, n - i);  // bytes of the chunk
  const uint8_t c = L < cl ? w.win[i + L - w.wb] : (uint8_t)0;
  const JWFrame F = st[d - 1];
  const bool in = L < cl;
  const uint64_t WS = __ballot(in && json_ws(c)), Q = __ballot(in && c == '"');
  const uint64_t BAD = __ballot(in && (c == '\\' || c < 0x20));  // escapes / control bytes end the fast path
  const uint64_t DG = __ballot(in && c >= '0' && c <= '9');
  const uint64_t valid = jw_range(0, cl);
  auto nonws = [&](uint32_t p) -> uint32_t {
    const uint64_t m = ~WS & valid & jw_from(p);
    return m ? (uint32_t)__builtin_ctzll(m) : 64u;
  };
  auto is = [&](uint32_t p, uint8_t ch) -> bool { return p < cl && (__ballot(in && c == ch) >> p) & 1ull; };
  uint32_t p = nonws(0);
  if (p >= cl) return 0;
  if (is(p, F.is_arr ? ']' : '}')) {  // the container's close
    uint32_t dn = 0;
    if (F.is_arr && F.count) {
      dn = dec_len(F.count);
      if (nb + 12 > g.cap_b || jb + dn > lim || nf >= g.cap_f) return 0;
      if (L == 0) {
        dec_put(F.count, dn, g.bytes + nb);
        Field f;
        f.k = g.bytes + F.koff;
        f.v = g.bytes + nb;
        f.kn = F.kn;
        f.vn = dn;
        f.kind = FK_ARG_POST;
        f._pad = F.h;
        g.fields[nf] = f;
      }
      nb += dn;
      jb += dn;
      nf++;
    }
    i += p + 1;
    d--;
    return 1;
  }
  if (F.count) {
    if (!is(p, ',')) return 0;
    p = nonws(p + 1);
    if (p >= cl) return 0;
  }
  uint32_t kn, ns = 0, dn = 0, v;
  if (!F.is_arr) {
    if (!jw_bit(Q, p)) return 0;
    ns = p + 1;
    const uint64_t mq = Q & jw_from(ns);
    if (!mq) return 0;
    const uint32_t qe = (uint32_t)__builtin_ctzll(mq);
    if (BAD & jw_range(ns, qe)) return 0;
    const uint32_t co = nonws(qe + 1);
    if (co >= cl || !is(co, ':')) return 0;
    v = nonws(co + 1);
    if (v >= cl) return 0;
    kn = F.kn + 1 + (qe - ns);
    if (nb + kn > g.cap_b) return 0;
  } else {
    v = p;
    dn = dec_len(F.count);
    kn = F.kn + 1 + dn;
    if (nb + F.kn + 12 > g.cap_b) return 0;
  }
  if (kn > GI_JW_PATH || jb + kn > lim) return 0;
  // the value: kind 0 container, 1 string, 2 number / literal; [vs, ve) its bytes, e = the chunk offset after it
  int kind;
  uint32_t vs = v, ve, e;
  bool arr = false;
  if (is(v, '{') || is(v, '[')) {
    if (d >= GI_JSON_MAX_DEPTH) return 0;
    kind = 0;
    arr = is(v, '[');
    ve = e = v + 1;
  } else if (jw_bit(Q, v)) {
    const uint64_t mq = Q & jw_from(v + 1);
    if (!mq) return 0;
    ve = (uint32_t)__builtin_ctzll(mq);
    if (BAD & jw_range(v + 1, ve)) return 0;
    kind = 1;
    vs = v + 1;
    e = ve + 1;
  } else if (is(v, 't') || is(v, 'f') || is(v, 'n')) {
    const uint32_t ln = is(v, 'f') ? 5u : 4u;
    const char* lit = is(v, 't') ? "true" : is(v, 'f') ? "false" : "null";
    if (v + ln > cl) return 0;
    const uint64_t ok = __ballot(L >= v && L < v + ln && c == (uint8_t)lit[L - v]);
    if (ok != jw_range(v, v + ln)) return 0;
    kind = 2;
    ve = is(v, 'n') ? v : v + ln;
    e = v + ln;
  } else {  // json_number_end over the masks
    auto nondig = [&](uint32_t a) -> uint32_t {
      const uint64_t m = ~DG & jw_from(a);
      return m ? (uint32_t)__builtin_ctzll(m) : 64u;
    };
    uint32_t x = v;
    if (is(x, '-')) x++;
    if (!jw_bit(DG, x)) return 0;
    x = is(x, '0') ? x + 1 : nondig(x);
    if (x < cl && is(x, '.')) {
      x++;
      if (!jw_bit(DG, x)) return 0;
      x = nondig(x);
    }
    if (x < cl && (is(x, 'e') || is(x, 'E'))) {
      x++;
      if (x < cl && (is(x, '+') || is(x, '-'))) x++;
      if (!jw_bit(DG, x)) return 0;
      x = nondig(x);
    }
    if (x >= cl) return 0;  // (it may go on past the chunk)
    kind = 2;
    ve = e = x;
  }
  if (kind != 0 && nf >= g.cap_f) return 0;
  // commit: the key (path + arena) and its hash, the frame count, the value
  const uint32_t koff = nb;
  uint32_t acc = 0;
  for (uint32_t j = L; j < kn; j += 64) {
    uint8_t b;
    if (j < F.kn) {
      b = path[j];
    } else if (j == F.kn) {
      b = '.';
    } else if (!F.is_arr) {
      b = w.win[i + ns + (j - F.kn - 1) - w.wb];
    } else {
      uint32_t x = F.count;
      for (uint32_t k = j - F.kn - 1; k + 1 < dn; k++) x /= 10;
      b = (uint8_t)('0' + x % 10);
    }
    g.bytes[koff + j] = b;
    if (j >= F.kn) path[j] = b;
    acc += jw_hmix(b, j);
  }
  const uint32_t kh = wave_sum(acc) ^ (kn * 0x27D4EB2Fu);
  nb += kn;
  jb += kn;
  if (L == 0) st[d - 1].count = F.count + 1;
  if (kind == 0) {
    if (L == 0) st[d] = {koff, kn, 0, arr ? 1u : 0u, kh};
    d++;
  } else {
    if (L == 0) {
      Field f;
      f.k = g.bytes + koff;
      f.v = q + i + vs;
      f.kn = kn;
      f.vn = ve - vs;
      f.kind = FK_ARG_POST;
      f._pad = kh;
      g.fields[nf] = f;
    }
    nf++;
  }
  i += e;
  return 1;
}

// Fields [nf0, *nf) and the arena [nb0, *nb) as parse_json_body(+ fold) makes
// them; false: no fields (not parsed here).
__device__ bool wave_parse_json(const Region& g, const uint8_t* q, uint32_t n, uint32_t nf0, uint32_t nb0,
                                gi_lds_u8* win, uint32_t W, gi_lds_u8* path, JWFrame* st, uint32_t* nf_out,
                                uint32_t* nb_out, unsigned long long* prof) {
  const uint32_t L = lane_id();
  const bool l0 = L == 0;
  JWin w{q, win, n, W, 0, 0, 0, 0};
  const bool fast = W >= 256;
  uint64_t pk = 0, pb = 0, pv = 0, pm = 0, c_0 = 0;  // GI_PROF: key, build, value cycles, members
  const uint64_t c_start = gi_clock();
  uint32_t nf = nf0, nb = nb0;
  uint32_t i = 0;
  while (i < n && json_ws(jw_at(w, i))) i++;
  if (i >= n || (jw_at(w, i) != '{' && jw_at(w, i) != '[')) return false;
  // the sequential parser's frame stack and root key allocations
  const uint32_t stn = (GI_JSON_MAX_DEPTH + 1) * sizeof(JFrame) + 8;
  if (nb + stn + 4 > g.cap_b) return false;
  nb += stn;
  const uint32_t root = nb;
  nb += 4;
  if (l0) {
    g.bytes[root] = 'j'; g.bytes[root + 1] = 's'; g.bytes[root + 2] = 'o'; g.bytes[root + 3] = 'n';
  }
  if (L < 4) path[L] = "json"[L];
  __syncthreads();
  uint32_t d = 1;
  const uint32_t h0 = wave_key_hash(path, 4);
  const uint32_t arr0 = jw_at(w, i) == '[' ? 1u : 0u;
  if (l0) st[0] = {root, 4, 0, arr0, h0};
  __syncthreads();
  const uint64_t lim = 4ull * n + 1024;
  uint64_t jb = 0;
  i++;
  auto add = [&](uint32_t koff, uint32_t kn, uint32_t h, const uint8_t* v, uint32_t vn) -> bool {
    if (nf >= g.cap_f) return false;
    if (l0) {
      Field f;
      f.k = g.bytes + koff;
      f.v = v;
      f.kn = kn;
      f.vn = vn;
      f.kind = FK_ARG_POST;
      f._pad = h;
      g.fields[nf] = f;
    }
    nf++;
    return true;
  };
  while (d > 0) {
    if (fast) {
      // one member (or element, or a container's close) read from 64 bytes of
      // the window at i with bit masks; 0: not that simple -- the member takes
      // the path below, which also decides every error
      const int r = jw_fast_member(g, w, q, i, d, nf, nb, jb, lim, path, st);
      if (r) {
        wave_lds_sync();  // path / st written
        continue;
      }
    }
    JWFrame F = st[d - 1];
    while (i < n && json_ws(jw_at(w, i))) i++;
    if (i >= n) return false;
    if (jw_at(w, i) == (F.is_arr ? ']' : '}')) {
      i++;
      if (F.is_arr && F.count) {
        if (nb + 12 > g.cap_b) return false;
        const uint32_t dn = dec_len(F.count);
        if (l0) dec_put(F.count, dn, g.bytes + nb);
        const uint32_t vo = nb;
        nb += dn;
        jb += dn;
        if (jb > lim) return false;
        if (!add(F.koff, F.kn, F.h, g.bytes + vo, dn)) return false;
      }
      d--;
      continue;
    }
    if (F.count) {
      if (jw_at(w, i) != ',') return false;
      i++;
      while (i < n && json_ws(jw_at(w, i))) i++;
    }
    // the element's key: the container's (path[0, F.kn)) + '.' + name / index
    uint32_t kn;
    const uint32_t koff = nb;
    if (prof) c_0 = gi_clock();
    if (F.is_arr) {
      if (nb + F.kn + 12 > g.cap_b) return false;
      const uint32_t dn = dec_len(F.count);
      kn = F.kn + 1 + dn;
      if (kn > GI_JW_PATH) return false;
      if (l0) {
        path[F.kn] = '.';
        dec_put(F.count, dn, path + F.kn + 1);
      }
      jb += kn;
      if (jb > lim) return false;
    } else {
      if (i >= n || jw_at(w, i) != '"') return false;
      bool esc;
      const uint32_t e = jw_string_end(w, i, &esc);
      if (!e) return false;
      const uint32_t rn = e - i - 2;
      if (nb + F.kn + 1 + rn > g.cap_b) return false;
      if (F.kn + 1 + rn > GI_JW_PATH) return false;
      if (L == 0) path[F.kn] = '.';
      uint32_t sn = rn;
      if (esc) {
        sn = jw_unescape(w, i + 1, rn, path + F.kn + 1, false);
      } else {
        jw_cover(w, i + 1, rn);
        for (uint32_t k = L; k < rn; k += 64) path[F.kn + 1 + k] = w.win[i + 1 + k - w.wb];
      }
      kn = F.kn + 1 + sn;
      jb += kn;
      if (jb > lim) return false;
      i = e;
      while (i < n && json_ws(jw_at(w, i))) i++;
      if (i >= n || jw_at(w, i) != ':') return false;
      i++;
      while (i < n && json_ws(jw_at(w, i))) i++;
    }
    uint64_t c_1 = prof ? gi_clock() : 0;
    wave_lds_sync();  // path written
    for (uint32_t k = L; k < kn; k += 64) g.bytes[koff + k] = path[k];
    const uint32_t kh = wave_key_hash(path, kn);
    nb += kn;
    uint64_t c_2 = prof ? gi_clock() : 0;
    F.count++;
    if (l0) st[d - 1].count = F.count;
    if (i >= n) return false;
    const uint8_t c = jw_at(w, i);
    if (c == '{' || c == '[') {
      if (d >= GI_JSON_MAX_DEPTH) return false;
      if (l0) st[d] = {koff, kn, 0, c == '[' ? 1u : 0u, kh};
      d++;
      i++;
    } else if (c == '"') {
      bool esc;
      const uint32_t e = jw_string_end(w, i, &esc);
      if (!e) return false;
      const uint32_t rn = e - i - 2;
      if (esc) {
        if (nb + rn > g.cap_b) return false;
        const uint32_t vo = nb;
        const uint32_t vn = jw_unescape(w, i + 1, rn, g.bytes + vo, true);
        nb += vn;
        jb += vn;
        if (jb > lim) return false;
        if (!add(koff, kn, kh, g.bytes + vo, vn)) return false;
      } else {
        if (!add(koff, kn, kh, q + i + 1, rn)) return false;
      }
      i = e;
    } else if (c == 't' || c == 'f' || c == 'n') {
      const uint32_t ln = c == 'f' ? 5 : 4;
      const char* lit = c == 't' ? "true" : c == 'f' ? "false" : "null";
      if (i + ln > n) return false;
      for (uint32_t k = 0; k < ln; k++)
        if (jw_at(w, i + k) != (uint8_t)lit[k]) return false;
      if (!add(koff, kn, kh, q + i, c == 'n' ? 0 : ln)) return false;
      i += ln;
    } else {
      const uint32_t e = jw_number_end(w, i);
      if (!e) return false;
      if (!add(koff, kn, kh, q + i, e - i)) return false;
      i = e;
    }
    wave_lds_sync();  // st written
    if (prof) {
      const uint64_t c_3 = gi_clock();
      pk += c_1 - c_0;
      pb += c_2 - c_1;
      pv += c_3 - c_2;
      pm++;
    }
  }
  while (i < n && json_ws(jw_at(w, i))) i++;
  if (i != n) return false;
  if (prof && l0) {
    atomicAdd(&prof[9], (unsigned long long)(gi_clock() - c_start));
    atomicAdd(&prof[10], (unsigned long long)w.rc);
    atomicAdd(&prof[11], (unsigned long long)w.nr);
    atomicAdd(&prof[12], (unsigned long long)pk);
    atomicAdd(&prof[13], (unsigned long long)pb);
    atomicAdd(&prof[14], (unsigned long long)pv);
    atomicAdd(&prof[15], (unsigned long long)pm);
    atomicAdd(&prof[16], 1ull);
  }
  // repeated keys (json_fold_keys: first position, last value)
  const uint32_t nk = nf - nf0;
  if (nk >= 2) {
    const uint32_t cap = g.cap_t / 4;
    if (nk >= cap) return false;
    uint32_t tsize = 16;
    while (tsize < 2 * nk && 2 * tsize <= cap) tsize *= 2;
    if (tsize > cap || tsize <= nk) tsize = cap;
    uint32_t* tab = (uint32_t*)g.t1;
    for (uint32_t k = L; k < tsize; k += 64) tab[k] = 0;
    __syncthreads();  // the table and the fields lane 0 wrote
    bool dup = false;
    for (uint32_t b = nf0; b < nf; b += 64) {
      const uint32_t fi = b + L;
      if (fi < nf) {
        const Field f = g.fields[fi];
        uint32_t s = f._pad % tsize;
        while (true) {
          const uint32_t old = atomicCAS(&tab[s], 0u, fi + 1);
          if (old == 0) break;
          const Field o = g.fields[old - 1];
          if (o._pad == f._pad && o.kn == f.kn && bytes_equal(o.k, f.k, f.kn)) {
            dup = true;
            break;
          }
          s = s + 1 == tsize ? 0 : s + 1;
        }
      }
    }
    if (__ballot(dup)) {
      __syncthreads();
      uint32_t res[2] = {0, 0};
      if (l0) {
        JsonCtx jc{g.fields, nf, g.cap_f, g.bytes, nb, g.cap_b, g.t1, g.cap_t, 0};
        json_fold_keys(jc, nf0);
        res[0] = jc.nf;
        res[1] = jc.flags;
      }
      nf = __shfl(res[0], 0, 64);
      if (__shfl(res[1], 0, 64)) return false;
    }
  }
  for (uint32_t k = nf0 + L; k < nf; k += 64) g.fields[k]._pad = 0;
  *nf_out = nf;
  *nb_out = nb;
  return true;
}

// ------------------------------------------------ wave urlencoded parse
// parse_query(body, ARGS_POST) for one wave, 4 KB of the body per step: lane
// L classifies bytes [64 L, 64 L + 64) of the step ('&', '=', '%' / '+' bit
// masks from aligned word loads), a segmented scan over the lanes carries the
// open segment (start, first '=', escapes before / after it) across lanes and
// steps, and each lane emits the fields of the segments its '&'s end, in body
// order (a wave prefix sum of the counts).  Keys / values with escapes decode
// into the arena at the segment's own body offset (a decoding is never longer
// than its input, so segments cannot collide), as before.
struct UrlSeg {
  uint32_t amp;  // start of the open segment (one past its '&')
  uint32_t eq;   // its first '=' (fl & 2)
  uint32_t fl;   // 1: the range holds an '&'; 2: the open segment has an '='; 4: '%' / '+' before its
                 // first '=' (anywhere, without one); 8: after it
};
__device__ __forceinline__ UrlSeg useg_cat(const UrlSeg& A, const UrlSeg& B) {
  if (B.fl & 1u) return B;
  UrlSeg R;
  R.amp = A.amp;
  R.fl = A.fl & 1u;
  if (A.fl & 2u) {
    R.eq = A.eq;
    R.fl |= 2u | (A.fl & 12u) | ((B.fl & 12u) ? 8u : 0u);
  } else if (B.fl & 2u) {
    R.eq = B.eq;
    R.fl |= 2u | (A.fl & 4u) | (B.fl & 12u);
  } else {
    R.eq = 0;
    R.fl |= (A.fl & 4u) | (B.fl & 4u);
  }
  return R;
}
// the summary of bits `rm` of a slice at body offset sb (no '&' among them)
__device__ __forceinline__ UrlSeg useg_range(uint64_t eqm, uint64_t escm, uint64_t rm, uint32_t sb) {
  UrlSeg S{0u, 0u, 0u};
  const uint64_t e = eqm & rm;
  if (e) {
    const uint32_t f = (uint32_t)__builtin_ctzll(e);
    S.eq = sb + f;
    const uint64_t below = (1ull << f) - 1ull;
    S.fl = 2u | ((escm & rm & below) ? 4u : 0u) | ((escm & rm & ~below & ~(1ull << f)) ? 8u : 0u);
  } else {
    S.fl = (escm & rm) ? 4u : 0u;
  }
  return S;
}
// zero bytes of x as a 4-bit mask
__device__ __forceinline__ uint32_t zbytes4(uint32_t x) {
  const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  const uint32_t z = ~nz & 0x80808080u;
  return ((z >> 7) | (z >> 14) | (z >> 21) | (z >> 28)) & 0xFu;
}

// Fields [nf0, *nf) for the urlencoded body q[0, n) (g.cap_b >= nb0 + n);
// false: more fields than the table holds
__device__ bool wave_parse_urlenc(const Region& g, const uint8_t* q, uint32_t n, uint32_t nf0, uint32_t nb0,
                                  uint32_t* nf_out, uint32_t* nb_out) {
  const uint32_t L = lane_id();
  UrlSeg C{0u, 0u, 1u};  // as if an '&' ended just before the body
  uint32_t nf = nf0, used = 0;
  const uint32_t s = (uint32_t)((uintptr_t)q & 3u);
  for (uint32_t wb = 0; wb < n; wb += 4096) {
    const uint32_t sb = wb + 64 * L;
    uint64_t amp = 0, eqm = 0, escm = 0;
    if (sb < n) {
      auto classify = [&](uint32_t x, uint32_t k) {
        amp |= (uint64_t)zbytes4(x ^ 0x26262626u) << (4 * k);
        eqm |= (uint64_t)zbytes4(x ^ 0x3D3D3D3Du) << (4 * k);
        escm |= (uint64_t)(zbytes4(x ^ 0x25252525u) | zbytes4(x ^ 0x2B2B2B2Bu)) << (4 * k);
      };
      if (sb + 68 <= n) {  // 17 aligned words hold the slice
        const uint32_t* pw = (const uint32_t*)(q + sb - s);
        uint32_t prev = pw[0];
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
          const uint32_t nxt = pw[k + 1];
          classify(s ? __builtin_amdgcn_alignbyte(nxt, prev, s) : prev, k);
          prev = nxt;
        }
      } else {
        for (uint32_t k = 0; k < 16; k++) {
          uint32_t x = 0;
          for (uint32_t b = 0; b < 4; b++)
            if (sb + 4 * k + b < n) x |= (uint32_t)q[sb + 4 * k + b] << (8 * b);
          classify(x, k);
        }
      }
      if (n - sb < 64) {  // (bytes past the body read as 0: no flags, but mask them anyway)
        const uint64_t vm = (1ull << (n - sb)) - 1ull;
        amp &= vm;
        eqm &= vm;
        escm &= vm;
      }
    }
    // this lane's summary: its tail after the last '&' (or the whole slice)
    UrlSeg S;
    if (amp) {
      const uint32_t last = 63u - (uint32_t)__builtin_clzll(amp);
      const uint64_t tm = last == 63 ? 0ull : ~0ull << (last + 1);
      S = useg_range(eqm, escm, tm, sb);
      S.fl |= 1u;
      S.amp = sb + last + 1;
    } else {
      S = useg_range(eqm, escm, ~0ull, sb);
      S.amp = 0;
    }
    // inclusive segmented scan over the lanes, then the open segment at this slice's start
    UrlSeg I = S;
    for (int o = 1; o < 64; o <<= 1) {
      UrlSeg Y;
      Y.amp = __shfl_up(I.amp, o, 64);
      Y.eq = __shfl_up(I.eq, o, 64);
      Y.fl = __shfl_up(I.fl, o, 64);
      if (L >= (uint32_t)o) I = useg_cat(Y, I);
    }
    UrlSeg X;
    X.amp = __shfl_up(I.amp, 1, 64);
    X.eq = __shfl_up(I.eq, 1, 64);
    X.fl = __shfl_up(I.fl, 1, 64);
    X = L == 0 ? C : useg_cat(C, X);
    UrlSeg T;
    T.amp = __shfl(I.amp, 63, 64);
    T.eq = __shfl(I.eq, 63, 64);
    T.fl = __shfl(I.fl, 63, 64);
    const UrlSeg Cn = useg_cat(C, T);
    // the non-empty segments this lane's '&'s end
    uint32_t cnt = 0;
    {
      uint32_t start = X.amp;
      for (uint64_t m = amp; m; m &= m - 1) {
        const uint32_t e = sb + (uint32_t)__builtin_ctzll(m);
        cnt += e > start ? 1u : 0u;
        start = e + 1;
      }
    }
    uint32_t tot;
    const uint32_t idx0 = nf + wave_excl_sum(cnt, &tot);
    if ((uint64_t)nf + tot + 1 > g.cap_f) return false;  // (+1: the body's last segment)
    uint32_t idx = idx0;
    UrlSeg O = X;
    uint32_t cur = 0;  // bit where the open segment's bytes in this slice begin
    for (uint64_t m = amp; m; m &= m - 1) {
      const uint32_t b = (uint32_t)__builtin_ctzll(m);
      const uint32_t e = sb + b;
      const uint64_t rm = (b > cur ? (~0ull >> (64 - (b - cur))) << cur : 0ull);
      const UrlSeg G = useg_cat(O, useg_range(eqm, escm, rm, sb));
      const uint32_t st = O.amp;
      if (e > st) {
        const bool he = G.fl & 2u;
        const uint8_t* k = q + st;
        uint32_t kn = (he ? G.eq : e) - st;
        const uint8_t* v = q + (he ? G.eq + 1 : e);
        uint32_t vn = he ? e - G.eq - 1 : 0;
        if (G.fl & 4u) {
          uint8_t* d = g.bytes + nb0 + st;
          kn = query_unescape(k, kn, d);
          k = d;
          used = max(used, st + kn);
        }
        if (G.fl & 8u) {
          const uint32_t vo = (uint32_t)(v - q);
          uint8_t* d = g.bytes + nb0 + vo;
          vn = query_unescape(v, vn, d);
          v = d;
          used = max(used, vo + vn);
        }
        Field f;
        f.k = k;
        f.v = v;
        f.kn = kn;
        f.vn = vn;
        f.kind = FK_ARG_POST;
        f._pad = 0;
        g.fields[idx++] = f;
      }
      O = UrlSeg{e + 1, 0u, 1u};
      cur = b + 1;
    }
    nf += tot;
    C = Cn;
  }
  // the body's last segment (no '&' after it)
  if (n > C.amp) {
    if (L == 0) {
      const uint32_t st = C.amp, e = n;
      const bool he = C.fl & 2u;
      const uint8_t* k = q + st;
      uint32_t kn = (he ? C.eq : e) - st;
      const uint8_t* v = q + (he ? C.eq + 1 : e);
      uint32_t vn = he ? e - C.eq - 1 : 0;
      if (C.fl & 4u) {
        uint8_t* d = g.bytes + nb0 + st;
        kn = query_unescape(k, kn, d);
        k = d;
        used = max(used, st + kn);
      }
      if (C.fl & 8u) {
        const uint32_t vo = (uint32_t)(v - q);
        uint8_t* d = g.bytes + nb0 + vo;
        vn = query_unescape(v, vn, d);
        v = d;
        used = max(used, vo + vn);
      }
      Field f;
      f.k = k;
      f.v = v;
      f.kn = kn;
      f.vn = vn;
      f.kind = FK_ARG_POST;
      f._pad = 0;
      g.fields[nf] = f;
    }
    nf++;
  }
  *nf_out = nf;
  *nb_out = nb0 + wave_max(used);
  return true;
}

#ifndef GI_BPARSE_WPE
#define GI_BPARSE_WPE 4  // k_bparse's register budget (waves per SIMD).  C3/C4 A/B: 4 (128 VGPRs, 30 spilled) 62 ms,
                         // 3 (168 VGPRs, no spills) 73 ms -- the parsers are latency chains, occupancy hides them
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GI_BPARSE_WPE))) k_bparse(DProgram P, DBatch B) {
  // JSON bodies up to B.bparse_lds bytes are parsed out of an LDS copy (the
  // sequential parser then waits on LDS, not on global memory, per byte)
  extern __shared__ __attribute__((aligned(16))) uint8_t jlds[];
  __shared__ uint32_t chist[2 * (GI_NCLS / 16)];  // item counts per class of this body's ARGS_POST values / keys
  __shared__ __attribute__((aligned(16))) uint8_t jpath[GI_JW_PATH];  // wave_parse_json's key path
  __shared__ JWFrame jst[GI_JSON_MAX_DEPTH + 1];                       // and frame stack
  const uint32_t L = threadIdx.x;
  for (uint32_t bi = blockIdx.x; bi < B.n_body; bi += gridDim.x) {
    const uint32_t r = B.body_list[bi];
    GI_BOUND(r < B.n_req, r, bi);
    if (B.stage == 2 && !B.pend[r]) continue;  // decided in phase 1 (wave-uniform)
    Region g = region_of(P, B, r);
    ReqHdr* H = g.hdr;
    const uint8_t sp = H->spec_proc;
    if ((sp != BP_URLENCODED && sp != BP_JSON) || (H->flags & GI_REQ_ERROR_MASK)) continue;  // multipart: k_mpparse
    const gi_span bs = B.reqs[r].body;
    const uint8_t* q = B.data + bs.off;
    const uint32_t n = bs.len;
    const uint32_t nf0 = H->nf, nb0 = H->nb;
    uint32_t n_post = 0, nb = nb0;
    bool ok = true;
    if (sp == BP_URLENCODED && (uint64_t)nb0 + n <= g.cap_b && B.bparse_wave) {
      uint32_t nfo = nf0;
      ok = wave_parse_urlenc(g, q, n, nf0, nb0, &nfo, &nb);
      n_post = nfo - nf0;
    } else if (sp == BP_URLENCODED && (uint64_t)nb0 + n <= g.cap_b) {
      const uint32_t a0 = (uint32_t)((uint64_t)n * L / 64), a1 = (uint32_t)((uint64_t)n * (L + 1) / 64);
      uint32_t c = 0;
      for (uint32_t p = a0; p < a1; p++) c += (q[p] != '&' && (p == 0 || q[p - 1] == '&')) ? 1u : 0u;
      uint32_t tot;
      uint32_t idx = nf0 + wave_excl_sum(c, &tot);
      n_post = tot;
      if ((uint64_t)nf0 + tot > g.cap_f) {
        ok = false;  // add_field would overflow
      } else {
        uint32_t used = 0;  // arena bytes [nb0, nb0 + used) this lane's decodings reach
        for (uint32_t p = a0; p < a1; p++) {
          if (q[p] == '&' || (p > 0 && q[p - 1] != '&')) continue;
          uint32_t j, e;
          bool kesc, vesc;
          urlenc_segment(q, n, p, &j, &e, &kesc, &vesc);
          const uint8_t* k = q + p;
          uint32_t kn = e - p;
          const uint8_t* v = q + (e < j ? e + 1 : j);
          uint32_t vn = e < j ? j - e - 1 : 0;
          if (kesc) {
            uint8_t* d = g.bytes + nb0 + p;
            kn = query_unescape(k, kn, d);
            k = d;
            used = max(used, p + kn);
          }
          if (vesc) {
            const uint32_t vo = (uint32_t)(v - q);
            uint8_t* d = g.bytes + nb0 + vo;
            vn = query_unescape(v, vn, d);
            v = d;
            used = max(used, vo + vn);
          }
          Field& f = g.fields[idx++];
          f.k = k;
          f.v = v;
          f.kn = kn;
          f.vn = vn;
          f.kind = FK_ARG_POST;
          f._pad = 0;
        }
        nb = nb0 + wave_max(used);
      }
    } else if (sp == BP_JSON && B.bparse_lds >= 2048 && B.bparse_wave) {
      // the body through an LDS window of B.bparse_lds bytes, the whole wave parsing
      uint32_t nfo = nf0;
      ok = wave_parse_json(g, q, n, nf0, nb0, (gi_lds_u8*)jlds, B.bparse_lds, (gi_lds_u8*)jpath,
                           jst, &nfo, &nb, B.prof);
      n_post = nfo - nf0;
      __syncthreads();  // the next body reuses the window
    } else {  // JSON (or an urlencoded body the arena bound does not cover): lane 0, sequential
      uint32_t res[3] = {0, 0, 0};
      if (L == 0) {
        if (sp == BP_URLENCODED) {
          Tx t;
          tx_bind(t, P, g);
          t.nf = nf0;
          t.nb = nb0;
          t.flags = 0;
          parse_query(t, q, n, FK_ARG_POST);
          res[0] = t.nf - nf0;
          res[1] = t.nb;
          res[2] = t.flags;
        }
      }
      const bool staged = sp == BP_JSON && n <= B.bparse_lds;
      if (staged) {  // the whole wave copies the body into LDS
        for (uint32_t k = L; k < n; k += 64) jlds[k] = q[k];
        __syncthreads();
      }
      if (L == 0 && sp == BP_JSON) {
        JsonCtx jc{g.fields, nf0, g.cap_f, g.bytes, nb0, g.cap_b, g.t1, g.cap_t, 0};
        parse_json_body(jc, staged ? jlds : q, n);
        res[0] = jc.nf - nf0;
        res[1] = jc.nb;
        res[2] = jc.flags;
      }
      n_post = __shfl(res[0], 0, 64);
      nb = __shfl(res[1], 0, 64);
      ok = __shfl(res[2], 0, 64) == 0;
      if (staged) {  // values that point into the LDS copy point into the body instead
        for (uint32_t k = L; k < n_post; k += 64) {
          Field& f = g.fields[nf0 + k];
          if (f.v >= jlds && f.v <= jlds + n) f.v = q + (f.v - jlds);
        }
        __syncthreads();  // the next body's copy overwrites jlds
      }
    }
    if (!ok) {  // not parsable as guessed: k_eval decides
      n_post = 0;
      nb = nb0;
    }
    __syncthreads();
    if (L == 0) {
      H->n_post = n_post;
      H->nb = nb;
      if (!ok) {
        H->spec_proc = BP_NONE;
        H->spec_err = 0;
        H->single[S_FILES_COMBINED_SIZE] = {CS_ZERO, 0};
      }
    }
    // phase-A item counts per length class of the body fields (ARGS_POST
    // sides some filter reads), aggregated in LDS
    const uint32_t sides = P.n_streams ? P.item_sides[FK_ARG_POST] : 0u;
    if (sides) {
      constexpr uint32_t NG = GI_NCLS / 16;
      for (uint32_t k = L; k < 2 * NG; k += 64) chist[k] = 0;
      __syncthreads();
      for (uint32_t i = L; i < n_post; i += 64) {
        const Field fl = g.fields[nf0 + i];
        if (fl.kind != FK_ARG_POST) continue;
        if (sides & 1) atomicAdd(&chist[item_class_in_group(fl.vn)], 1u);
        if (sides & 2) atomicAdd(&chist[NG + item_class_in_group(fl.kn)], 1u);
      }
      __syncthreads();
      for (uint32_t k = L; k < 2 * NG; k += 64)
        if (chist[k])
          atomicAdd(&B.bcounts[(r / 256) * GI_NCLS + item_class_of_group((FK_ARG_POST << 1) | (k / NG), k % NG)],
                    chist[k]);
      __syncthreads();
    }
  }
}

// Speculative multipart ProcessRequestBody: one workgroup per body.  Its
// threads first list every '\n' + "--" + boundary position of the body (each
// scans 1/GI_MP_T, a prefix sum orders the lists) into the request's t0
// buffer; the parts are then parsed in parallel (block_multipart) or, when
// that is not exact, by thread 0 alone with the sequential parser (Go
// mime/multipart restated), whose part-data delimiter search walks the list.
// On failure the request keeps no fields (k_eval parses it again).
#define GI_MP_MAX_BOUNDARY 256

// The body's parts split over the block's GI_MP_T threads: the delimiters
// are the candidates with '\r' before them that Go's matchAfterPrefix accepts
// (V); the part ending at V[j] starts at the delimiter line V[j - 1] + 1, and
// the first V entry whose line is the final delimiter ends the last part.
// Thread T parses parts [a, b) with the sequential parse_multipart itself,
// started at its first part's delimiter line and stopped at the next
// thread's, into its own slice of the t1 scratch (fields) and of the arena;
// the slices are then concatenated in thread order -- the order, and the
// allocations, of one sequential pass.  Anything a thread cannot reproduce
// exactly (an error, a segment that does not end where the next begins, a
// file name two threads both size, a quota overflow) returns false: thread 0
// then parses the body alone.  Every return is block-uniform.
#define GI_MP_T 256
struct MpShared {
  uint32_t wsum[GI_MP_T / 64];
  uint32_t used[GI_MP_T], bo[GI_MP_T];
  uint32_t res[5];
  uint32_t f, nfs;
  unsigned long long comb;
};

// exclusive prefix sum over the block (every thread calls it)
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t x, uint32_t* total, uint32_t* wsum) {
  const uint32_t W = threadIdx.x >> 6;
  uint32_t wt;
  const uint32_t e = wave_excl_sum(x, &wt);
  if ((threadIdx.x & 63) == 0) wsum[W] = wt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (uint32_t w = 0; w < GI_MP_T / 64; w++) {
    const uint32_t v = wsum[w];
    off += w < W ? v : 0u;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return off + e;
}

__device__ bool block_multipart(const Region& g, const uint8_t* s, uint32_t n, Str ct, const uint8_t* sbd, uint32_t bn,
                                uint32_t* cand, uint32_t ncand, uint32_t nf0, uint32_t nb0, MpShared& sh) {
  const uint32_t T = threadIdx.x;
  if (8ull * ncand > g.cap_t || g.cap_b <= nb0) return false;
  uint32_t* V = cand + ncand;
  // V: the delimiters, in body order
  uint32_t nv = 0;
  for (uint32_t c0 = 0; c0 < ncand; c0 += GI_MP_T) {
    const uint32_t c = c0 + T;
    bool v = false;
    if (c < ncand) {
      const uint32_t k = cand[c];
      v = k >= 1 && s[k - 1] == '\r' && mp_after_ok(s, n, k + 3 + bn);
    }
    uint32_t tot;
    const uint32_t at = block_excl_sum(v ? 1u : 0u, &tot, sh.wsum);
    if (v) V[nv + at] = cand[c];
    nv += tot;
  }
  // f: the first delimiter whose line is the final one
  if (T == 0) sh.f = 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t j0 = 0; j0 < nv; j0 += GI_MP_T) {
    const uint32_t j = j0 + T;
    if (j < nv) {
      const uint32_t ls = V[j] + 1;
      uint32_t e = ls + 2 + bn;
      while (e < n && e < ls + 2 + bn + 64 && s[e] != '\n') e++;
      if (e < n && s[e] == '\n') e++;
      if ((e >= n || s[e - 1] == '\n') && mp_is_final(s, ls, e, sbd, bn, false)) atomicMin(&sh.f, j);
    }
    __syncthreads();
    const bool found = sh.f != 0xFFFFFFFFu;
    __syncthreads();  // (everyone read it before the next round's atomicMin)
    if (found) break;
  }
  const uint32_t f = sh.f;
  if (f == 0xFFFFFFFFu) return false;
  const uint32_t np = f + 1;  // parts
  const uint32_t nl = min((uint32_t)GI_MP_T, np);
  const uint32_t fq = g.cap_t / (uint32_t)sizeof(Field) / GI_MP_T;  // fields per thread
  const uint32_t aq = ((g.cap_b - nb0) / GI_MP_T) & ~7u;            // arena bytes per thread
  uint32_t err = MP_OK, cnt = 0, used = 0;
  uint64_t comb = 0;
  bool cset = false, good = true;
  if (T < nl) {
    const uint32_t a = (uint32_t)((uint64_t)np * T / nl), b = (uint32_t)((uint64_t)np * (T + 1) / nl);
    const uint32_t i0 = a == 0 ? 0u : V[a - 1] + 1;
    const uint32_t stop = b == np ? 0xFFFFFFFFu : V[b - 1] + 1;
    if (a > 0) {  // a thread after the first starts at a plain "--boundary\r\n" line
      good = i0 + 4 + bn <= n && s[i0] == '-' && s[i0 + 1] == '-' && s[i0 + 2 + bn] == '\r' && s[i0 + 3 + bn] == '\n';
      for (uint32_t q = 0; q < bn && good; q++) good = s[i0 + 2 + q] == sbd[q];
    }
    if (good) {
      Field* fl = (Field*)g.t1 + (uint64_t)T * fq;
      JsonCtx jc{fl, 0, fq, g.bytes, nb0 + T * aq, nb0 + (T + 1) * aq, nullptr, 0, 0};
      uint32_t seg[2] = {0, 0};
      err = parse_multipart(jc, s, n, ct.p, ct.n, &comb, &cset, cand, ncand, i0, stop, seg);
      good = jc.flags == 0 && seg[0] == b - a && (b == np ? err == MP_OK : (err == MP_SEG && seg[1] == stop));
      cnt = jc.nf;
      used = jc.nb - (nb0 + T * aq);
    }
  }
  if (__syncthreads_or(!good)) return false;
  uint32_t ftot, btot;
  const uint32_t fo = block_excl_sum(cnt, &ftot, sh.wsum);
  const uint32_t bo = block_excl_sum(used, &btot, sh.wsum);
  if ((uint64_t)nf0 + ftot > g.cap_f) return false;
  sh.used[T] = used;
  sh.bo[T] = bo;
  if (T == 0) sh.comb = 0;
  __syncthreads();
  // the arena slices, moved down in thread order: through the t0 scratch
  // after V when it holds them all (every thread its own slice), else slice
  // by slice by the whole block (a forward copy: dst <= src)
  if (8ull * ncand + btot <= g.cap_t) {
    uint8_t* tmp = (uint8_t*)(V + ncand);
    for (uint32_t k = 0; k < used; k++) tmp[bo + k] = g.bytes[nb0 + T * aq + k];
    __syncthreads();
    for (uint32_t k = T; k < btot; k += GI_MP_T) g.bytes[nb0 + k] = tmp[k];
  } else {
    for (uint32_t l2 = 0; l2 < nl; l2++) {
      const uint32_t u2 = sh.used[l2], src = nb0 + l2 * aq, dst = nb0 + sh.bo[l2];
      if (src == dst) continue;
      for (uint32_t k0 = 0; k0 < u2; k0 += GI_MP_T) {
        uint8_t x = 0;
        if (k0 + T < u2) x = g.bytes[src + k0 + T];
        __syncthreads();
        if (k0 + T < u2) g.bytes[dst + k0 + T] = x;
        __syncthreads();
      }
    }
  }
  // the fields, in thread order, arena pointers rebased
  if (cnt) {
    const Field* fl = (const Field*)g.t1 + (uint64_t)T * fq;
    const uint8_t* lo = g.bytes + nb0 + T * aq;
    const uint8_t* hi = lo + aq;
    const uint64_t shift = (uint64_t)T * aq - bo;
    for (uint32_t i = 0; i < cnt; i++) {
      Field x = fl[i];
      if (x.k >= lo && x.k < hi) x.k -= shift;
      if (x.v >= lo && x.v < hi) x.v -= shift;
      g.fields[nf0 + fo + i] = x;
    }
  }
  if (comb) atomicAdd(&sh.comb, (unsigned long long)comb);
  __syncthreads();
  // FILES_SIZES: one entry per file name (eq_ascii_ci_both) across the
  // threads: the entries listed in LDS, then compared pairwise
  if (T == 0) sh.nfs = 0;
  __syncthreads();
  for (uint32_t i = nf0 + T; i < nf0 + ftot; i += GI_MP_T)
    if (g.fields[i].kind == FK_FILE_SIZE) {
      const uint32_t k = atomicAdd(&sh.nfs, 1u);
      if (k < GI_MP_T) sh.used[k] = i;
    }
  __syncthreads();
  const uint32_t nfs = sh.nfs;
  if (nfs > GI_MP_T) return false;
  bool dup = false;
  for (uint32_t a = T; a < nfs * nfs; a += GI_MP_T) {
    const uint32_t i = a / nfs, j = a % nfs;
    if (j >= i) continue;
    const Field x = g.fields[sh.used[i]], y = g.fields[sh.used[j]];
    if (y.kn == x.kn && eq_ascii_ci_both(y.k, x.k, x.kn)) dup = true;
  }
  if (__syncthreads_or(dup)) return false;
  const bool cs = __syncthreads_or(cset) != 0;
  if (T == 0) {
    const uint64_t ctot = sh.comb;
    sh.res[0] = MP_OK;
    sh.res[1] = nf0 + ftot;
    sh.res[2] = nb0 + btot;
    sh.res[3] = (uint32_t)ctot;
    sh.res[4] = (uint32_t)(ctot >> 32) | (cs ? 0x80000000u : 0u);
  }
  __syncthreads();
  return true;
}

__global__ void __launch_bounds__(GI_MP_T) k_mpparse(DProgram P, DBatch B) {
  __shared__ uint8_t sbd[GI_MP_MAX_BOUNDARY];
  __shared__ uint32_t sbn;
  __shared__ MpShared sh;
  const uint32_t T = threadIdx.x;
  for (uint32_t bi = blockIdx.x; bi < B.n_body; bi += gridDim.x) {
    const uint32_t r = B.body_list[bi];
    GI_BOUND(r < B.n_req, r, bi);
    if (B.stage == 2 && !B.pend[r]) continue;  // decided in phase 1 (block-uniform)
    Region g = region_of(P, B, r);
    ReqHdr* H = g.hdr;
    if (H->spec_proc != BP_MULTIPART || (H->flags & GI_REQ_ERROR_MASK)) continue;  // block-uniform
    const gi_span bs = B.reqs[r].body;
    const uint8_t* s = B.data + bs.off;
    const uint32_t n = bs.len;
    const uint32_t nf0 = H->nf, nb0 = H->nb;
    const Str ct = first_content_type(B, B.reqs[r]);
    __syncthreads();  // (every thread read H before thread 0 rewrites it below)
    if (T == 0) {  // the boundary (a throw-away arena copy: parse_multipart parses the media type again)
      JsonCtx jc{g.fields, nf0, g.cap_f, g.bytes, nb0, g.cap_b, g.t1, g.cap_t, 0};
      uint32_t ts, te;
      Str bstr;
      sbn = 0;
      if (mp_media(jc, ct.p, ct.n, &ts, &te, "boundary", &bstr, nullptr, nullptr) == 0 && bstr.n > 0 &&
          bstr.n <= GI_MP_MAX_BOUNDARY) {
        for (uint32_t k = 0; k < bstr.n; k++) sbd[k] = bstr.p[k];
        sbn = bstr.n;
      }
    }
    __syncthreads();
    const uint32_t bn = sbn;
    uint32_t* cand = (uint32_t*)g.t0;
    uint32_t ncand = 0;
    bool use = false;
    if (bn) {
      const uint32_t a0 = (uint32_t)((uint64_t)n * T / GI_MP_T), a1 = (uint32_t)((uint64_t)n * (T + 1) / GI_MP_T);
      auto hit = [&](uint32_t k) {
        if (s[k] != '\n' || k + 3 + bn > n || s[k + 1] != '-' || s[k + 2] != '-') return false;
        for (uint32_t q = 0; q < bn; q++)
          if (s[k + 3 + q] != sbd[q]) return false;
        return true;
      };
      // the '\n' bytes of the slice from aligned words, then the full test at each
      auto scan = [&](uint32_t* out, uint32_t at) {
        uint32_t c = 0;
        uint32_t k = a0;
        for (; k < a1 && ((uintptr_t)(s + k) & 3u); k++)
          if (hit(k)) {
            if (out) out[at + c] = k;
            c++;
          }
        for (; k + 4 <= a1; k += 4) {
          for (uint32_t m = zbytes4(*(const uint32_t*)(s + k) ^ 0x0A0A0A0Au); m; m &= m - 1) {
            const uint32_t kk = k + (uint32_t)__builtin_ctz(m);
            if (hit(kk)) {
              if (out) out[at + c] = kk;
              c++;
            }
          }
        }
        for (; k < a1; k++)
          if (hit(k)) {
            if (out) out[at + c] = k;
            c++;
          }
        return c;
      };
      const uint32_t c = scan(nullptr, 0);
      uint32_t tot;
      const uint32_t at = block_excl_sum(c, &tot, sh.wsum);
      use = 4ull * tot <= g.cap_t;
      if (use) scan(cand, at);
      ncand = tot;
    }
    __syncthreads();
    // the part-parallel parse (block_multipart), else thread 0 alone
    bool done = false;
    if (use && ncand && B.mp_wave) done = block_multipart(g, s, n, ct, sbd, bn, cand, ncand, nf0, nb0, sh);
    if (!done) {
      if (T == 0) {
        JsonCtx jc{g.fields, nf0, g.cap_f, g.bytes, nb0, g.cap_b, g.t1, g.cap_t, 0};
        uint64_t comb;
        bool comb_set;
        const uint8_t err = parse_multipart(jc, s, n, ct.p, ct.n, &comb, &comb_set, use ? cand : nullptr, use ? ncand : 0u);
        sh.res[0] = jc.flags ? 0xFFu : err;
        sh.res[1] = jc.nf;
        sh.res[2] = jc.nb;
        sh.res[3] = (uint32_t)comb;
        sh.res[4] = (uint32_t)(comb >> 32) | (comb_set ? 0x80000000u : 0u);
      }
      __syncthreads();
    }
    uint32_t res[5];
    for (int k = 0; k < 5; k++) res[k] = sh.res[k];
    __syncthreads();  // (sh.res is rewritten below)
    bool ok = res[0] != 0xFFu;
    uint32_t nfe = res[1], nbe = res[2];
    if (T == 0 && ok && (res[4] >> 31)) {
      const uint64_t comb = (uint64_t)res[3] | ((uint64_t)(res[4] & 0x7FFFFFFFu) << 32);
      if (nbe + 24 > g.cap_b) {
        ok = false;
      } else {
        uint8_t* cb = g.bytes + nbe;
        const uint32_t cn2 = go_itoa((int64_t)comb, cb);
        nbe += cn2;
        H->single[S_FILES_COMBINED_SIZE] = {cb, cn2};
      }
    }
    if (T == 0) {
      sh.res[0] = ok;
      sh.res[1] = nbe;
    }
    __syncthreads();
    ok = sh.res[0] != 0;
    nbe = sh.res[1];
    if (!ok) {  // an engine limit / unsupported input: k_eval decides
      if (T == 0) H->spec_proc = BP_NONE;
    } else {
      if (T == 0) {
        H->spec_err = (uint8_t)res[0];
        H->n_post = nfe - nf0;
        H->nb = nbe;
      }
      // phase-A item counts per length class of its ARGS_POST and FILES*
      // fields (for_each_item's kinds)
      if (P.n_streams) {
        for (uint32_t f = nf0 + T; f < nfe; f += GI_MP_T) {
          const Field fl = g.fields[f];
          if (fl.kind < FK_ARG_GET || fl.kind > FK_FILE_SIZE) continue;
          const uint32_t sides = P.item_sides[fl.kind];
          if (sides & 1) atomicAdd(&B.bcounts[(r / 256) * GI_NCLS + item_class(fl.kind, 0, fl.vn)], 1u);
          if (sides & 2) atomicAdd(&B.bcounts[(r / 256) * GI_NCLS + item_class(fl.kind, 1, fl.kn)], 1u);
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------- header dedup
// A chunk's requests repeat most header lines byte for byte (User-Agent,
// Accept*, Host, ...), and phase A's results for a (field kind, side, key,
// value) are the same wherever it occurs: the filters admitting it depend on
// the kind, side and key, the chains, automata, validators and detectors on
// the bytes.  k_collect keys every header side by its bytes in a chunk-wide
// table: the first occurrence claims the entry (the canonical one, scanned as
// usual), a later byte-equal one becomes no item at all (Field._pad bit
// `side`).  After phase A, k_dspread gives each such copy the canonical
// value's results: its value-signature word, and per slot of that signature
// the exact / maybe key of the canonical's hit set -> hit bit + the copy's own
// hit-set key.  Exact: a canonical whose results are not exactly known (its
// hit set overflowed, its request voided or flagged) voids the copy's request
// (k_eval then evaluates it in full).  Nobody waits: an entry seen before its
// claimer published it just leaves this occurrence canonical-less (scanned).
#define GI_HD_PROBES 16
// (a word at a time: header bytes sit in the padded request arena)
__device__ __forceinline__ unsigned long long hdr_mix(unsigned long long h, const uint8_t* p, uint32_t n) {
  h = (h ^ (0x100000000ull | n)) * 1099511628211ull;
  for (uint32_t i = 0; i < n; i += 4) {
    uint32_t w = load_u32u(p + i);
    if (n - i < 4) w &= (1u << (8 * (n - i))) - 1u;
    h = (h ^ w) * 1099511628211ull;
  }
  return h;
}
__device__ __forceinline__ unsigned long long hdr_hash(uint32_t side, const Field& f) {
  unsigned long long h = hdr_mix((1469598103934665603ull ^ (side + 1u)) * 1099511628211ull, f.k, f.kn);
  if (side == 0) h = hdr_mix(h, f.v, f.vn);
  return h | 1ull;
}
__device__ __forceinline__ bool hdr_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  bool eq = true;
  for (uint32_t i = 0; i < n && eq; i += 4) {
    uint32_t x = load_u32u(a + i) ^ load_u32u(b + i);
    if (n - i < 4) x &= (1u << (8 * (n - i))) - 1u;
    eq = x == 0;
  }
  return eq;
}
__device__ __forceinline__ bool hdr_same(uint32_t side, const Field& a, const Field& b) {
  if (a.kn != b.kn || (side == 0 && a.vn != b.vn)) return false;
  return hdr_eq(a.k, b.k, a.kn) && (side != 0 || hdr_eq(a.v, b.v, a.vn));
}
// Entry info word, published once with one 64-bit atomic store: (global
// header index + 1) << 37 | request << 13 | (field * 2 + side).  A reader
// compares its bytes with the canonical's through the global header record
// and the request arena -- input data, immutable -- so it needs no acquire
// ordering (and pays no cache invalidation) to trust what it compares.
#define GI_HD_INFO(g, r, fs) ((((unsigned long long)(g) + 1ull) << 37) | ((unsigned long long)(r) << 13) | (fs))
__device__ __forceinline__ uint32_t hd_info_req(unsigned long long inf) { return (uint32_t)(inf >> 13) & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t hd_info_fs(unsigned long long inf) { return (uint32_t)inf & 0x1FFFu; }
__device__ __forceinline__ uint32_t hd_info_hdr(unsigned long long inf) { return (uint32_t)(inf >> 37) - 1u; }

// The canonical occurrence of header side (f, side) of request r (global
// header index g, field fi): true with its entry when a published byte-equal
// entry exists; otherwise an empty entry on the way is claimed (this
// occurrence becomes canonical).
__device__ bool hdr_find(const DBatch& B, unsigned long long h, uint32_t side, const Field& f, uint32_t r, uint32_t fi,
                         uint32_t g, uint32_t* ent) {
  const bool can_claim = g + 1u < (1u << 27) && r < (1u << 24) && 2u * fi + side < (1u << 13);
  for (uint32_t p = 0; p < GI_HD_PROBES; p++) {
    const uint32_t e = (uint32_t)(h + p) & B.hdmask;
    unsigned long long k = __atomic_load_n(&B.hdkeys[e], __ATOMIC_RELAXED);
    if (k == 0) {
      if (!can_claim) return false;
      k = atomicCAS(&B.hdkeys[e], 0ull, h);
      if (k == 0) {
        atomicExch(&B.hdinfo[e], GI_HD_INFO(g, r, 2u * fi + side));
        return false;
      }
    }
    if (k != h) continue;
    const unsigned long long inf = __atomic_load_n(&B.hdinfo[e], __ATOMIC_RELAXED);
    if (inf == 0) return false;  // not published yet: this occurrence stays canonical-less
    if ((hd_info_fs(inf) & 1u) != side || hd_info_req(inf) == r) continue;
    const gi_header hd = B.headers[hd_info_hdr(inf)];
    Field c;
    c.k = B.data + hd.name.off;
    c.kn = hd.name.len;
    c.v = B.data + hd.value.off;
    c.vn = hd.value.len;
    if (!hdr_same(side, f, c)) continue;
    *ent = e;
    return true;
  }
  return false;
}
// (a copy's canonical entry + 1 goes to hdref[2 * global header index + side]:
// k_dspread reads it instead of probing again)
__device__ void hdr_dedup(const DProgram& P, const DBatch& B, uint32_t r, const ReqHdr* H, Field* Fd) {
  const uint32_t sides = P.item_sides[FK_HEADER];
  const gi_request rq = B.reqs[r];
  uint32_t hx = 0;  // header record of field i (collect_request skips empty names)
  for (uint32_t i = H->n_get; i < H->n_get + H->n_hdr; i++) {
    while (hx < rq.hdr_count && B.headers[rq.hdr_begin + hx].name.len == 0) hx++;
    const uint32_t g = rq.hdr_begin + hx++;
    const Field fl = Fd[i];
    uint32_t mark = 0;
    for (uint32_t side = 0; side < 2; side++) {
      if (!((sides >> side) & 1u)) continue;
      uint32_t e;
      if (hdr_find(B, hdr_hash(side, fl), side, fl, r, i, g, &e)) {
        mark |= 1u << side;
        B.hdref[2ull * g + side] = e + 1u;
      }
    }
    Fd[i]._pad = mark;
  }
}

// ProcessURI + AddRequestHeader* for one request per thread, then the
// per-block item counts per length bucket (k_ioffsets / k_items) and the hit
// bits of links without an automaton image.
__global__ void __launch_bounds__(256) k_collect(DProgram P, DBatch B) {
  __shared__ uint32_t hist[GI_NCLS];
  for (uint32_t k = threadIdx.x; k < GI_NCLS; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B.n_req) {
    collect_request(P, B, r);
    if (P.n_streams) {
      const ReqLayout L = B.layout[r];
      const ReqHdr* H = (const ReqHdr*)(B.scratch + L.base);
      if (!(H->flags & GI_REQ_ERROR_MASK)) {
        Field* Fd = (Field*)(B.scratch + L.base + GI_REQHDR_BYTES);
        if (B.hdkeys) hdr_dedup(P, B, r, H, Fd);
        for_each_item(P, H, Fd,
                      [&](uint8_t kind, uint8_t, uint32_t side, uint32_t, uint32_t n) {
                        atomicAdd(&hist[item_class(kind, side, n)], 1u);
                      }, 0u, B.hdkeys != nullptr);
      }
      for (uint32_t k = 0; k < P.n_always; k++) set_hit(B, P.always_slots[k], r);
    }
  }
  __syncthreads();
  if (P.n_streams)
    for (uint32_t k = threadIdx.x; k < GI_NCLS; k += blockDim.x) B.bcounts[blockIdx.x * GI_NCLS + k] = hist[k];
}


// The gate's body stage (launch_pipeline): per-block item counts of the body
// fields of the pending requests (k_collect's layout: one thread per request,
// 256 per block).
__global__ void __launch_bounds__(256) k_bcounts(DProgram P, DBatch B) {
  __shared__ uint32_t hist[GI_NCLS];
  for (uint32_t k = threadIdx.x; k < GI_NCLS; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B.n_req && B.pend[r]) {
    const ReqLayout L = B.layout[r];
    const ReqHdr* H = (const ReqHdr*)(B.scratch + L.base);
    if (!(H->flags & GI_REQ_ERROR_MASK))
      for_each_item(P, H, (const Field*)(B.scratch + L.base + GI_REQHDR_BYTES),
                    [&](uint8_t kind, uint8_t, uint32_t side, uint32_t, uint32_t n) {
                      atomicAdd(&hist[item_class(kind, side, n)], 1u);
                    }, 2u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < GI_NCLS; k += blockDim.x) B.bcounts[blockIdx.x * GI_NCLS + k] = hist[k];
}

// ============================================================== phase A
// Data-parallel operator evaluation (SURVEY §2 rx_dfa_scan / ac_scan /
// simple_ops).  Every rule link whose operator is a pure function of one
// transformed value (@rx, @pm, @contains literal, @validate*) and whose
// targets are immutable request variables gets a hit slot; phase A sets the
// slot's bit for a request iff some admitted value matches (negated operators:
// iff some admitted value does not).  A clear bit proves the link cannot
// match, so k_eval skips it; a set bit is re-evaluated exactly by k_eval.
//
//   k_collect  fields per request + per-block item counts per length bucket
//   k_ioffsets bucket bases + per-block offsets (one workgroup)
//   k_items    item records (one per scanned (field, side) / single) into
//              length-bucketed ranges
//   k_stream   lane per item, wave per 64 items of one bucket: for every
//              stream (transformation chain) the item's admitting filters are
//              looked up in its global-filter mask, the chain runs once in
//              lane-private LDS buffers, validate operators are evaluated, and
//              the admitted values of the wave are written as ONE transposed
//              queue block (word w of lane i at w * nv + i: coalesced reads)
//   k_scan     LDS-resident automata images; a wave steps all automata of its
//              job in lockstep over the 64 values of one queue block
//   k_scan_slow non-ASCII values (rune decoding) and transformation
//              overflows, on the global tables
struct Item {  // 32 B
  const uint8_t* kp;  // key (fields); nullptr for singles
  const uint8_t* vp;  // scanned bytes: value side, key side or single
  uint32_t kn, vn;
  uint32_t req;
  uint32_t meta;      // bits 0-2 FieldKind (0 = single); fields: bit 3 key side (the *_NAMES
                      // collections), bits 4-31 field index; singles: bits 8-15 SingleId
};
static_assert(sizeof(Item) == 32, "Item layout");
#define GI_MAX_ITEM_FIELD 0x0FFFFFFFu
__device__ __forceinline__ uint32_t item_kind(const Item& it) { return it.meta & 7u; }
__device__ __forceinline__ uint32_t item_side(const Item& it) { return (it.meta >> 3) & 1u; }
__device__ __forceinline__ uint32_t item_single(const Item& it) { return (it.meta >> 8) & 0xFFu; }
// value-map index of the item (2 x field + side); GI_NO_VIX for singles
#define GI_NO_VIX 0xFFFFFFFFu
__device__ __forceinline__ uint32_t meta_vix(uint32_t meta) {
  return (meta & 7u) ? 2u * (meta >> 4) + ((meta >> 3) & 1u) : GI_NO_VIX;
}

// A scanned value set hit bit `slot` of request r: the bit, and the value's
// bit in the request's value map (k_eval tests only mapped values of the
// links whose slot is value-exact, see eval_rule).
__device__ __forceinline__ void hit_value(const DBatch& B, uint32_t slot, uint32_t r, uint32_t vix, uint32_t maybe = 0) {
  set_hit(B, slot, r);
  if (vix != GI_NO_VIX) {
    const ReqLayout L = B.layout[r];
    GI_BOUND(vix < L.vmap_bits, vix, L.vmap_bits);
    atomicOr(&B.vmap[L.vmap_bit + vix], 1u << (slot & 31));  // the value's slot signature
    if (L.hset_mask) hset_insert(B, L, slot, vix, maybe);
  }
}
// the same for the item at global index idx (k_scan's queue lanes carry it)
__device__ __forceinline__ void hit_item(const DBatch& B, uint32_t slot, uint32_t idx) {
  GI_BOUND(idx < B.items_cap, idx, B.items_cap);
  const uint2 rm = *(const uint2*)((const uint8_t*)B.items + 32ull * idx + 24);  // (req, meta)
  hit_value(B, slot, rm.x, meta_vix(rm.y));
}

// One workgroup per length class: the class's per-block item counts
// bcounts[blk * GI_NCLS + c] -> per-block offsets within the class (boffs),
// and the class total (ctot[c]).
__global__ void __launch_bounds__(256) k_ioffsets(DBatch B, uint32_t n_blocks) {
  __shared__ uint32_t part[256];
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint32_t chunk = (n_blocks + 255) / 256;
  const uint32_t k0 = min(n_blocks, t * chunk), k1 = min(n_blocks, (t + 1) * chunk);
  uint32_t sum = 0;
  for (uint32_t k = k0; k < k1; k++) sum += B.bcounts[k * GI_NCLS + c];
  part[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive scan
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t k = k0; k < k1; k++) {
    const uint32_t x = B.bcounts[k * GI_NCLS + c];
    B.boffs[k * GI_NCLS + c] = run;
    run += x;
  }
  if (t == 255) B.ctot[c] = part[255];
}

// Class bases (bucket-major order), bucket (base, count), item-wave base per
// bucket and the total: one workgroup scans the class totals.
__global__ void __launch_bounds__(256) k_ibases(DBatch B) {
  __shared__ uint32_t part[256];
  const uint32_t t = threadIdx.x;
  constexpr uint32_t per = (GI_NCLS + 255) / 256;
  const uint32_t c0 = min(GI_NCLS, t * per), c1 = min(GI_NCLS, (t + 1) * per);
  uint32_t sum = 0;
  for (uint32_t c = c0; c < c1; c++) sum += B.ctot[c];
  part[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t c = c0; c < c1; c++) {
    B.cbase[c] = run;
    run += B.ctot[c];
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t total = part[255];
    uint32_t iw = 0;
    for (uint32_t b = 0; b < GI_NB; b++) {
      const uint32_t lo = B.cbase[kClsBase[b]];
      const uint32_t hi = kClsBase[b + 1] < GI_NCLS ? B.cbase[kClsBase[b + 1]] : total;
      B.ibk[2 * b] = lo;
      B.ibk[2 * b + 1] = hi - lo;
      atomicAdd(&B.acct3[b], (unsigned long long)(hi - lo));
      B.ibk[2 * GI_NB + b] = iw;
      iw += (hi - lo + 63) / 64;
    }
    B.ibk[3 * GI_NB] = iw;
  }
}

// One thread per request, same block shape as k_collect.
__global__ void __launch_bounds__(256) k_items(DProgram P, DBatch B) {
  __shared__ uint32_t rank[GI_NCLS];
  __shared__ unsigned long long ibytes[GI_NB];
  for (uint32_t k = threadIdx.x; k < GI_NCLS; k += blockDim.x) rank[k] = 0;
  if (threadIdx.x < GI_NB) ibytes[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B.n_req && (B.stage != 2 || B.pend[r])) {
    const ReqLayout L = B.layout[r];
    const ReqHdr* H = (const ReqHdr*)(B.scratch + L.base);
    if (!(H->flags & GI_REQ_ERROR_MASK)) {
      const Field* Fd = (const Field*)(B.scratch + L.base + GI_REQHDR_BYTES);
      const uint32_t* boff = B.boffs + blockIdx.x * GI_NCLS;
      for_each_item(P, H, Fd, [&](uint8_t kind, uint8_t sg, uint32_t side, uint32_t fi, uint32_t n) {
        const uint32_t b = item_bucket(n), c = item_class(kind, side, n);
        const uint32_t at = B.cbase[c] + boff[c] + atomicAdd(&rank[c], 1u);
        GI_BOUND(at < B.items_cap, at, B.items_cap);
        Item it;
        if (kind == 0) {
          it.kp = nullptr;
          it.kn = 0;
          it.vp = H->single[sg].p;
        } else {
          const Field fl = Fd[fi];
          it.kp = fl.k;
          it.kn = fl.kn;
          it.vp = side ? fl.k : fl.v;
        }
        it.vn = n;
        it.req = r;
        it.meta = kind ? (uint32_t)kind | (side << 3) | (min(fi, GI_MAX_ITEM_FIELD) << 4) : (uint32_t)sg << 8;
        if (kind && fi > GI_MAX_ITEM_FIELD) void_request(B, r, GI_VOID_FIELD);  // no value-map index: no phase-A bit trusted
        ((Item*)B.items)[at] = it;
        atomicAdd(&ibytes[b], (unsigned long long)n);
      }, B.stage == 2 ? 2u : 0u, B.hdkeys != nullptr);  // the body stage: the pending requests' body fields
    }
  }
  __syncthreads();
  if (threadIdx.x < GI_NB && ibytes[threadIdx.x]) atomicAdd(&B.acct[threadIdx.x], ibytes[threadIdx.x]);
}

// Global filters admitting the item (bit g of the result).
__device__ uint64_t item_gmask(const DProgram& P, const Item& it) {
  uint64_t m = 0;
  // key hashes (read the key once): literal selectors / exceptions compare
  // bytes only on a hash hit
  const uint32_t kind = item_kind(it);
  const uint32_t hci = kind ? gi_fnv1a(it.kp, it.kn, true) : 0u;
  const uint32_t hcs = kind ? gi_fnv1a(it.kp, it.kn, false) : 0u;
  for (uint32_t g = 0; g < P.n_gfilters; g++) {
    const DFilter F = gi_cload(P.filters, g);
    if (kind == 0) {
      if (F.single == item_single(it)) m |= 1ull << g;
      continue;
    }
    if (F.single != GI_NO_SINGLE || !((F.kind_mask >> kind) & 1) || F.names != item_side(it)) continue;
    if (F.key_mode == 1) {
      if ((F.ci ? hci : hcs) != F.key_hash) continue;
      if (F.ci ? !eq_ascii_ci(it.kp, it.kn, P.strpool + F.key_off, F.key_len)
               : !eq_bytes(it.kp, it.kn, P.strpool + F.key_off, F.key_len))
        continue;
    } else if (F.key_mode == 2) {
      if (!dfa_match(P, F.key_dfa, it.kp, it.kn, F.ci != 0)) continue;
    }
    bool ex = false;
    for (uint32_t e = 0; e < F.exc_count && !ex; e++) {
      const DExc x = P.excs[F.exc_begin + e];
      ex = x.dfa >= 0 ? dfa_match(P, x.dfa, it.kp, it.kn, true)
                      : (hci == x.hash && eq_ascii_ci(it.kp, it.kn, P.strpool + x.off, x.len));
    }
    if (!ex) m |= 1ull << g;
  }
  return m;
}

// The stream's validate operators (@validateByteRange / UrlEncoding / Utf8Encoding).
// @detectSQLi / @detectXSS candidate (k_stream -> k_detect): the value bytes
// are copied to the detect arena; `mask` = the detect streams (DStream.det_id)
// whose vals test this value (several when chains left it unchanged).
struct DetEnt {
  uint32_t req, vix, mask, len;
  uint64_t off, gm;  // arena byte offset; the item's global filter mask
};

// every detect val of the masked streams that admits the value (gm): its bit
// becomes "maybe" (list overflow: exact, k_eval re-evaluates)
__device__ void det_maybe(const DProgram& P, const DBatch& B, uint32_t r, uint32_t vix, uint64_t gm, uint32_t mask) {
  for (uint32_t d = 0; d < P.n_det_streams; d++) {
    if (!((mask >> d) & 1u)) continue;
    const DStream S = P.streams[P.det_streams[d]];
    const uint64_t fm = gm & S.gmask;
    for (uint32_t q = 0; q < S.val_count; q++) {
      const DScanVal& sv = P.svals[S.val_begin + q];
      if ((sv.kind == OP_DETECT_SQLI || sv.kind == OP_DETECT_XSS) && (fm & sv.fmask)) hit_value(B, sv.slot, r, vix, 1u);
    }
  }
}

// Called by the whole wave (uniform control flow); lanes with `push` list
// their value.  One leader lane reserves the wave's entries and bytes (two
// atomics per wave instead of two per candidate on the same two counters).
__device__ void det_push(const DProgram& P, const DBatch& B, bool push, uint32_t r, uint32_t vix, uint64_t gm,
                         uint32_t mask, const uint8_t* v, uint32_t n) {
  const uint64_t am = __ballot(push);
  if (!am) return;
  uint32_t btot;
  const uint32_t boff = wave_excl_sum(push ? (n + 15) & ~15u : 0u, &btot);
  const int leader = __ffsll((unsigned long long)am) - 1;
  uint32_t k0 = 0;
  unsigned long long o0 = 0;
  if (lane_id() == (uint32_t)leader) {
    k0 = atomicAdd(B.det_count, (uint32_t)__popcll(am));
    o0 = atomicAdd(B.det_used, (unsigned long long)btot);
  }
  k0 = (uint32_t)__shfl((int)k0, leader, 64);
  o0 = ((unsigned long long)(uint32_t)__shfl((int)(uint32_t)(o0 >> 32), leader, 64) << 32) |
       (uint32_t)__shfl((int)(uint32_t)o0, leader, 64);
  if (!push) return;
  const uint32_t k = k0 + mask_rank(am);
  const unsigned long long off = o0 + boff;
  if (k >= B.det_cap || off + n > B.det_bytes_cap) {
    det_maybe(P, B, r, vix, gm, mask);
    return;
  }
  copy_bytes(B.det_bytes + off, v, n);
  DetEnt e;
  e.req = r;
  e.vix = vix;
  e.mask = mask;
  e.len = n;
  e.off = off;
  e.gm = gm;
  ((DetEnt*)B.det)[k] = e;
}

// The stream's scan values on its output v[0, n): validate operators here;
// @detectSQLi/@detectXSS through their exact prefilters -- a value that cannot
// match is settled (a negated val hits), a candidate goes to k_detect: once
// per item for the unchanged (raw) value (*rawmask collects the streams),
// else once for this stream's output (*det_append).
__device__ void stream_vals(const DProgram& P, const DBatch& B, uint32_t r, uint32_t vix, const DStream& S, uint64_t fm,
                            bool maybe, const uint8_t* v, uint32_t n, uint32_t osum, bool raw, uint32_t* rawmask,
                            bool* det_append, bool body) {
  for (uint32_t q = 0; q < S.val_count; q++) {
    const DScanVal sv = gi_cload(P.svals, S.val_begin + q);  // wave-uniform: scalar loads
    if (!(fm & sv.fmask) || !stage_runs(B, body, sv.prefix)) continue;
    if (sv.kind == OP_DETECT_SQLI || sv.kind == OP_DETECT_XSS) {
      if (maybe) {
        hit_value(B, sv.slot, r, vix, 1u);
        continue;
      }
      // the output's byte summary carries the exact prefilters (li_sqli_byte / li_xss_byte)
      const bool cand = (osum & (sv.kind == OP_DETECT_SQLI ? BS_LI_SQLI : BS_LI_XSS)) != 0;
      if (!cand) {
        if (sv.negate) hit_value(B, sv.slot, r, vix);
        continue;
      }
      if (raw) *rawmask |= 1u << S.det_id;
      else *det_append = true;
      continue;
    }
    if (maybe) hit_value(B, sv.slot, r, vix, 1u);
    else if (validate_op(sv.kind, sv.bits, v, n) != (sv.negate != 0)) hit_value(B, sv.slot, r, vix);
  }
}

// chain through two buffers of capacity cap; -1 on overflow.  summ = byte
// summary of v: transformations it proves to be identities are skipped.
template <bool INL>
__device__ __forceinline__ int64_t run_chain(const DProgram& P, const DStream& S, const uint8_t* v, uint32_t vn,
                                             uint32_t summ, uint8_t* b0, uint8_t* b1, uint32_t cap,
                                             const uint8_t** out, const uint16_t* lut, uint32_t* osumm) {
  const uint8_t* cur = v;
  uint32_t cn = vn;
  for (uint32_t k = 0; k < S.tchain_len; k++) {
    const uint8_t code = (uint8_t)GI_CONST(uint32_t, P.tchains32)[S.tchain_off + k];
    if (transform_identity(summ, code)) continue;
    uint8_t* dst = (cur == b0) ? b1 : b0;
    const int64_t m = INL ? apply_transform_inl(P, code, cur, cn, dst, cap) : apply_transform(P, code, cur, cn, dst, cap);
    if (m < 0) return -1;
    cur = dst;
    cn = (uint32_t)m;
    summ = value_summary_lut(lut, cur, cn);
  }
  *out = cur;
  *osumm = summ;  // byte summary of the output (k_stream's LUT adds the libinjection prefilter bits)
  return cn;
}

// Per-item memo of chain results (k_stream, short buckets).  Different
// streams' chains reduce to the same few effective chains on most values:
// the identity steps drop out (e.g. t:urlDecodeUni on a value without '%'),
// and what remains -- t:cmdLine, t:lowercase, ... -- repeats across streams.
// A lane keeps the last M outputs of the current item keyed by the effective
// code sequence applied so far (1, then key * 64 + code), and a chain resumes
// from the longest memoised prefix instead of recomputing it.
struct ChainMemo {
  uint64_t key;
  uint32_t len, sum;
};
template <uint32_t M, uint32_t WT>
__device__ __forceinline__ int64_t run_chain_memo(const DProgram& P, const DStream& S, const uint8_t* v, uint32_t vn,
                                                  uint32_t summ, uint8_t* slots, ChainMemo* memo, uint32_t* victim,
                                                  uint8_t* b0, uint8_t* b1, const uint8_t** out, const uint16_t* lut,
                                                  uint32_t* osumm) {
  const uint8_t* cur = v;
  uint32_t cn = vn, cur_slot = M;  // M: cur is not a memo slot
  uint64_t key = 1;
  for (uint32_t k = 0; k < S.tchain_len; k++) {
    const uint8_t code = (uint8_t)GI_CONST(uint32_t, P.tchains32)[S.tchain_off + k];
    if (transform_identity(summ, code)) continue;
    key = key * 64u + code;
    uint32_t hit = M;
    for (uint32_t m = 0; m < M; m++)
      if (memo[m * 64].key == key) hit = m;
    if (hit < M) {
      cur_slot = hit;
      cur = slots + hit * 64u * WT;
      cn = memo[hit * 64].len;
      summ = memo[hit * 64].sum;
      continue;
    }
    uint32_t vs = *victim;
    if (vs == cur_slot) vs = (vs + 1) % M;
    uint8_t* dst;
    if (vs == cur_slot) {  // M == 1 and the input is the slot: the scratch buffers, not memoised
      dst = cur == b0 ? b1 : b0;
      vs = M;
    } else {
      *victim = (vs + 1) % M;
      dst = slots + vs * 64u * WT;
    }
    const int64_t m = apply_transform_inl(P, code, cur, cn, dst, WT);
    if (m < 0) return -1;
    cur = dst;
    cur_slot = vs;
    cn = (uint32_t)m;
    summ = value_summary_lut(lut, cur, cn);
    if (vs < M) memo[vs * 64] = ChainMemo{key, cn, summ};
  }
  *out = cur;
  *osumm = summ;
  return cn;
}

// Slow-list entry: the transformed bytes are copied into the slow arena.
struct SlowEnt {
  uint32_t req, stream, flags, len;  // flags: bit0 maybe
  uint32_t vix, _pad;                // value-map index (GI_NO_VIX: a single)
  uint64_t off;                      // byte offset in B.slow_bytes
  uint64_t fm;                       // admitting filters (global ids)
};

// Collapse a value for a stream whose automata map every non-ASCII rune to one
// class: each rune >= 0x80 (a valid UTF-8 sequence, or one invalid byte that
// utf8.DecodeRune reads as U+FFFD) becomes one GI_RUNE_MARK byte, so the
// lockstep scan steps exactly once per rune, as the rune-decoding scan does.
// With a rune map (DStream.rmap_cnt > 0: the automata tell some non-ASCII
// runes apart) each rune becomes 0x80 + its joint class instead.
__device__ uint32_t collapse_runes(const uint8_t* s, uint32_t n, uint8_t* d, const uint32_t* rmap, uint32_t rcnt) {
  uint32_t o = 0;
  for (uint32_t i = 0; i < n;) {
    if (s[i] < 0x80) {
      d[o++] = s[i++];
    } else {
      uint32_t w;
      const uint32_t r = decode_rune(s, n, i, &w);
      i += w;
      uint8_t b = GI_RUNE_MARK;
      if (rcnt) {
        uint32_t lo = 0, hi = rcnt;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (rmap[mid * 3 + 1] < r) lo = mid + 1;
          else hi = mid;
        }
        if (lo < rcnt && rmap[lo * 3] <= r) b = (uint8_t)rmap[lo * 3 + 2];
      }
      d[o++] = b;
    }
  }
  return o;
}

// IN = per-lane LDS copy of the item's bytes (bucket maximum); WT = per-lane
// LDS transformation buffers.  IN == 0: long items, HBM buffers throughout.
// 2 waves/SIMD: the chains + queue writer fit without spills (at 3 the
// compiler spilled ~128 VGPRs, and scratch traffic dominated k_stream's HBM
// writes: PMC WRITE_SIZE 38 GB per launch against 4.6 GB of queue words)
#ifndef GI_STREAM_WPE
#define GI_STREAM_WPE 2
#endif
template <uint32_t IN, uint32_t WT, uint32_t M>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GI_STREAM_WPE, 8))) k_stream(DProgram P, DBatch B, uint32_t bucket) {
  constexpr uint32_t IS = IN ? IN + 4 : 0;  // lane strides = odd dword counts: conflict-free
  __shared__ __attribute__((aligned(16))) uint8_t lb[IN ? 64 * (IS + (2 + M) * WT) : 16];
  __shared__ ChainMemo memo_s[M ? 64 * M : 1];  // [slot][lane]
  // Queue block of (item-wave, stream) = qblk[stream][item-wave index]: no
  // counter.  Pool words are reserved GI_PCHUNK at a time per wave (one
  // workgroup = one wave), so the pool counter sees one atomic per chunk.
  __shared__ unsigned long long pnext, pend;
  __shared__ uint16_t sumlut[256];  // byte_summary of every byte value
  const uint32_t lane = threadIdx.x;
  if (lane == 0) pnext = pend = 0;
  for (uint32_t b = lane; b < 256; b += 64)
    sumlut[b] = (uint16_t)(byte_summary((uint8_t)b) | (li_sqli_byte((uint8_t)b) ? BS_LI_SQLI : 0u) |
                           (li_xss_byte((uint8_t)b) ? BS_LI_XSS : 0u));
  __syncthreads();
  const uint32_t iw_base = B.ibk[2 * GI_NB + bucket];
  const uint32_t base = B.ibk[2 * bucket], cnt = B.ibk[2 * bucket + 1];
  uint8_t* g0 = B.lscratch + ((uint64_t)blockIdx.x * 64 + lane) * 2ull * B.lcap;
  uint8_t* g1 = g0 + B.lcap;
  uint8_t* li = IN ? lb + lane * IS : nullptr;
  uint8_t* b0 = IN ? lb + 64 * IS + lane * WT : g0;
  uint8_t* b1 = IN ? lb + 64 * (IS + WT) + lane * WT : g1;
  uint8_t* mslots = lb + 64 * (IS + 2 * WT) + lane * WT;  // memo slot m of this lane at mslots + m * 64 * WT
  ChainMemo* memo = memo_s + lane;
  uint32_t victim = 0;
  const uint32_t cap = IN ? WT : B.lcap;
  uint64_t pc_item = 0, pc_chain = 0, pc_out = 0, pc_loop = 0, pc_tot = 0, pc_fm = 0, pc_run = 0, pc_slow = 0;
  uint64_t pc_vals = 0, pc_det = 0;
  uint64_t wwords = 0;  // queue words this wave wrote (algorithmic-byte accounting)
  uint64_t csteps = 0;  // value bytes this lane fed into a stream's chain (secondary roofline)
  const uint64_t pc_start = B.prof ? gi_clock() : 0;
  for (uint32_t w0 = blockIdx.x * 64; w0 < cnt; w0 += gridDim.x * 64) {
    const uint64_t c_a = B.prof ? gi_clock() : 0;
    const uint32_t ii = w0 + lane;
    for (uint32_t m = 0; m < M; m++) memo[m * 64].key = 0;  // a new item: nothing memoised
    Item it{};
    uint64_t gm = 0;
    const uint8_t* src = nullptr;
    uint32_t summ = 0;
    if (ii < cnt) {
      GI_BOUND(base + ii < B.items_cap, base + ii, B.items_cap);
      it = ((const Item*)B.items)[base + ii];
      GI_BOUND(it.req < B.n_req, it.req, ii);
      gm = item_gmask(P, it);
      B.igm[base + ii] = gm;  // k_scan's per-lane filter mask (the queue lanes carry the item index)
      src = it.vp;
      if (IN) {  // stage the scanned bytes once for all streams (bucket: vn <= IN): the
        // aligned words covering the value, all loads in flight at once (<= 3 bytes past its
        // end: padded sources)
        const uint32_t n = min(it.vn, IN);
        const uintptr_t a = (uintptr_t)it.vp;
        const uint32_t sh = (uint32_t)(a & 3u);
        const uint32_t* wp = (const uint32_t*)(a - sh);
        const uint32_t nw = (sh + n + 3) / 4;
        uint32_t wv[IN / 4 + 1];
#pragma unroll
        for (uint32_t k = 0; k < IN / 4 + 1; k++) wv[k] = k < nw ? wp[k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < IN / 4; k++)
          if (4 * k < n) *(uint32_t*)(li + 4 * k) = sh ? __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], sh) : wv[k];
        src = li;
      }
      summ = value_summary_lut(sumlut, src, it.vn);
    }
    const uint32_t blk = iw_base + w0 / 64;
    const uint64_t c_b = B.prof ? gi_clock() : 0;
    pc_item += c_b - c_a;
    // Blocks whose every value left its chain unchanged hold the raw item
    // bytes: a later stream with the same lane set points its qblk entry at
    // the earlier block instead of writing it again (the lane header carries
    // the stream-independent filter mask gm; each job's fmask table ignores
    // filters of other streams).
    uint64_t rom0 = 0, rom1 = 0;
    uint32_t rq0 = 0, rq1 = 0, rw0 = 0, rw1 = 0;
    uint32_t rawmask = 0;  // detect streams whose output is the unchanged item (one k_detect entry per item)
    // a long value (>= GI_LONG_MIN bytes) takes k_long: one wave per (item, stream), no queue block
    const bool is_long = IN == 0 && B.long_cap && ii < cnt && it.vn >= GI_LONG_MIN;
    // the gate (launch_pipeline): the first stage scans body fields through the
    // prefix streams only, the body stage through the others
    const uint32_t ik = item_kind(it);
    const bool body_item = ik == FK_ARG_POST || (ik >= FK_FILE && ik <= FK_FILE_SIZE);
    for (uint32_t s = 0; s < P.n_streams; s++) {
      const uint64_t c_s0 = B.prof ? gi_clock() : 0;
      const DStream S = gi_cload(P.streams, s);
      const bool skip_s = B.stage == 1 && body_item && !S.prefix;
      const uint64_t fm0 = skip_s ? 0ull : gm & S.gmask;
      if (is_long && fm0) {
        const uint32_t k = atomicAdd(B.long_count, 1u);
        if (k < B.long_cap) B.long_list[k] = make_uint2(base + ii, s);
        else void_request(B, it.req, GI_VOID_LONG);  // list full: the request's phase-A bits are void (exact)
      }
      const uint64_t fm = is_long ? 0ull : fm0;
      if (!__ballot(fm != 0)) {
        if (lane == 0 && S.job_count && blk < B.qcap) B.qblk[(uint64_t)s * B.qcap + blk] = make_uint2(0u, 0u);
        continue;
      }
      const uint64_t c_sa = B.prof ? gi_clock() : 0;
      pc_fm += c_sa - c_s0;
      const uint8_t* cur = nullptr;
      int64_t cn = 0;
      bool det_append = false;  // this stream's output is a @detectSQLi/@detectXSS candidate (k_detect)
      uint32_t osum = summ;  // byte summary of the chain output
      bool maybe = false, glob = !IN;
      if (fm) {
        csteps += it.vn;
        if (M) cn = run_chain_memo<M, WT>(P, S, src, it.vn, summ, mslots, memo, &victim, b0, b1, &cur, sumlut, &osum);
        else cn = run_chain<IN != 0>(P, S, src, it.vn, summ, b0, b1, cap, &cur, sumlut, &osum);
        if (B.prof) pc_run += gi_clock() - c_sa;
        if (cn < 0 && IN) {
          cn = run_chain<false>(P, S, src, it.vn, summ, g0, g1, B.lcap, &cur, sumlut, &osum);
          glob = true;
        }
        if (cn < 0) {
          maybe = true;
          cur = src;
          cn = 0;
        }
        const uint64_t c_v0 = B.prof ? gi_clock() : 0;
        if (S.val_count)
          stream_vals(P, B, it.req, meta_vix(it.meta), S, fm, maybe, cur, (uint32_t)cn, osum, !maybe && cur == src,
                      &rawmask, &det_append, body_item);
        if (B.prof) pc_vals += gi_clock() - c_v0;
      }
      const uint64_t c_d0 = B.prof ? gi_clock() : 0;
      if (S.val_count) det_push(P, B, det_append, it.req, meta_vix(it.meta), gm, 1u << S.det_id, cur, (uint32_t)cn);
      if (B.prof) pc_det += gi_clock() - c_d0;
      const uint64_t c_s1 = B.prof ? gi_clock() : 0;
      pc_chain += c_s1 - c_s0;
      if (!S.job_count) continue;
      bool slow = maybe;
      if (fm && !maybe) {
        // byte summary of the chain output (run_chain leaves it current in
        // the identity case; recompute otherwise)

        if (osum & BS_HIGH) {
          if (S.collapse) {
            uint8_t* dst = glob ? (cur == g0 ? g1 : g0) : (cur == b0 ? b1 : b0);
            cn = collapse_runes(cur, (uint32_t)cn, dst, P.nranges + S.rmap_off, S.rmap_cnt);
            cur = dst;
          } else {
            slow = true;
          }
        }
      }
      if (fm && slow) {  // per-value path (k_scan_slow)
        const uint32_t k = atomicAdd(B.slow_count, 1u);
        const unsigned long long off = atomicAdd(B.slow_used, (unsigned long long)((cn + 15) & ~15ll));
        if (k >= B.slow_cap || off + (uint64_t)cn > B.slow_bytes_cap) {
          void_request(B, it.req, GI_VOID_SLOW);
        } else {
          copy_bytes(B.slow_bytes + off, cur, (uint32_t)cn);
          SlowEnt e;
          e.req = it.req;
          e.stream = s;
          e.fm = fm;
          e.flags = (maybe ? 1u : 0u) | (body_item ? 2u : 0u);
          e.vix = meta_vix(it.meta);
          e._pad = 0;
          e.off = off;
          e.len = (uint32_t)cn;
          ((SlowEnt*)B.slow)[k] = e;
        }
      }
      const uint64_t c_s2 = B.prof ? gi_clock() : 0;
      pc_slow += c_s2 - c_s1;
      const bool out = fm && !slow;
      const uint64_t om = __ballot(out);
      if (!om) {
        if (lane == 0 && blk < B.qcap) B.qblk[(uint64_t)s * B.qcap + blk] = make_uint2(0u, 0u);
        continue;
      }
      const uint32_t nv = __popcll(om);
      const uint32_t nw = wave_max(out ? ((uint32_t)cn + 3) / 4 : 0u);
      const uint32_t qbody = __ballot(out && !body_item) ? 0u : GI_QB_BODY;  // (a wave may straddle kinds)
      const bool raw = __ballot(out && cur != src) == 0;  // every output is the staged item
      if (raw && (om == rom0 || om == rom1)) {
        if (lane == 0 && blk < B.qcap)
          B.qblk[(uint64_t)s * B.qcap + blk] = om == rom0 ? make_uint2(rw0, rq0) : make_uint2(rw1, rq1);
        continue;
      }
      // blocks start on 16-byte cells: qblk holds the cell index (64 GB of pool)
      const uint64_t words = ((uint64_t)nv * (GI_QB_HDR + nw) + 3) & ~3ull;
      unsigned long long woff = 0;
      wwords += (uint64_t)nv * (GI_QB_HDR + nw);
      if (lane == 0) {
        if (pnext + words > pend) {
          const unsigned long long sz = words > GI_PCHUNK ? words : (unsigned long long)GI_PCHUNK;
          const unsigned long long b0p = atomicAdd(B.pool_used, sz);
          pnext = b0p;
          pend = b0p + sz;
        }
        woff = pnext;
        pnext += words;
      }
      woff = __shfl(woff, 0, 64);
      if (blk >= B.qcap || woff + words > B.pool_cap) {  // out of queue space: exact fallback
        if (out) void_request(B, it.req, blk >= B.qcap ? GI_VOID_QCAP : GI_VOID_POOL);
        if (lane == 0 && blk < B.qcap) B.qblk[(uint64_t)s * B.qcap + blk] = make_uint2(0u, 0u);
        continue;
      }
      if (lane == 0) B.qblk[(uint64_t)s * B.qcap + blk] = make_uint2((uint32_t)(woff >> 2), nv | (nw << 8) | qbody);
      if (raw) {  // remember it (two most recent lane sets)
        rom1 = rom0, rq1 = rq0, rw1 = rw0;
        rom0 = om, rq0 = nv | (nw << 8) | GI_QB_SHARED | qbody, rw0 = (uint32_t)(woff >> 2);
      }
      if (out) {
        const uint32_t i = mask_rank(om);
        uint32_t* q = B.pool + woff;
        q[i] = base + ii;  // global item index: k_scan reaches the filter mask (B.igm) and, on a hit,
                           // (req, value-map index) through it
        q[nv + i] = (uint32_t)cn;
        const uint32_t nwi = ((uint32_t)cn + 3) / 4;
        if (IN && !glob) {  // cur is a lane buffer in LDS (dword-aligned): a word per read
          for (uint32_t w = 0; w < nwi; w++) {
            uint32_t x = ((const uint32_t*)cur)[w];
            if (4 * w + 4 > (uint32_t)cn) x &= (1u << (8 * ((uint32_t)cn - 4 * w))) - 1u;
            q[GI_QB_HDR * nv + (uint64_t)w * nv + i] = x;
          }
        } else {  // cur in HBM (the item value or a lane's global buffer, both padded): a word per read
          for (uint32_t w = 0; w < nwi; w++)
            q[GI_QB_HDR * nv + (uint64_t)w * nv + i] = load_u32u(cur + 4 * w) & tail_mask((uint32_t)cn - 4 * w);
        }
      }
      if (B.prof) pc_out += gi_clock() - c_s2;
    }
    det_push(P, B, rawmask != 0, it.req, meta_vix(it.meta), gm, rawmask, src, it.vn);
    if (B.prof) pc_loop += gi_clock() - c_b;
  }
  if (lane == 0 && wwords) atomicAdd(&B.acct[5 + bucket], (unsigned long long)wwords);
  csteps = wave_sum(csteps);
  if (lane == 0 && csteps) atomicAdd(&B.acct2[bucket], (unsigned long long)csteps);
  if (B.prof && lane == 0) {
    pc_tot = gi_clock() - pc_start;
    gi_prof_add(&B.prof[40 + 5 * bucket + 0], (unsigned long long)pc_item);
    gi_prof_add(&B.prof[40 + 5 * bucket + 1], (unsigned long long)pc_chain);
    gi_prof_add(&B.prof[40 + 5 * bucket + 2], (unsigned long long)pc_out);
    gi_prof_add(&B.prof[40 + 5 * bucket + 3], (unsigned long long)pc_loop);
    gi_prof_add(&B.prof[40 + 5 * bucket + 4], (unsigned long long)pc_tot);
    gi_prof_add(&B.prof[80 + 3 * bucket + 0], (unsigned long long)pc_fm);
    gi_prof_add(&B.prof[80 + 3 * bucket + 1], (unsigned long long)pc_run);
    gi_prof_add(&B.prof[80 + 3 * bucket + 2], (unsigned long long)pc_slow);
    gi_prof_add(&B.prof[24 + 2 * bucket], (unsigned long long)pc_vals);
    gi_prof_add(&B.prof[25 + 2 * bucket], (unsigned long long)pc_det);
  }
}

__device__ __forceinline__ uint32_t rune_class(const DProgram& P, const DDfa& d, uint32_t r) {
  if (d.nonascii_uniform) return d.nonascii_cls;
  const uint32_t* nr = P.nranges + d.nr_off;
  uint32_t lo = 0, hi = d.nr_cnt;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (nr[mid * 3 + 1] < r) lo = mid + 1;
    else hi = mid;
  }
  return (lo < d.nr_cnt && nr[lo * 3] <= r) ? nr[lo * 3 + 2] : 0u;
}

// Bit k of the result: pattern k of the automaton matches somewhere in s
// (global tables; rune decoding exactly like utf8.DecodeRune).
__device__ uint64_t scan_full(const DProgram& P, const DDfa& d, const uint8_t* s, uint32_t n) {
  const uint16_t* tr = P.trans + d.trans_off;
  const uint8_t* amap = P.u8pool + d.amap_off;
  const uint8_t* combo = P.u8pool + d.combo_off;
  const uint32_t ncls = d.n_classes;
  uint32_t st = d.start;
  uint64_t m = 0;
  const uint64_t* acc = P.u64pool + d.acc_off;
  for (uint32_t i = 0; i < n;) {
    if (!d.multi && st == d.accept) return 1;
    const uint8_t c = s[i];
    uint32_t cls;
    if (d.byte_mode || c < 0x80) {
      cls = amap[c];
      i++;
    } else {
      uint32_t w;
      const uint32_t rr = decode_rune(s, n, i, &w);
      i += w;
      cls = rune_class(P, d, rr);
    }
    const uint32_t tv = tr[st * ncls + cls];
    if (d.multi) {
      if (tv & 0x8000) m |= acc[(uint64_t)st * 5 + combo[cls]];
      st = tv & 0x7FFF;
    } else {
      st = tv;
    }
  }
  if (d.multi) return m | acc[(uint64_t)st * 5 + 4];
  return P.u8pool[d.endacc_off + st] ? 1ull : 0ull;
}

// Per-value path on global tables: every automaton of job J over one value.
__device__ void scan_value_global(const DProgram& P, const DBatch& B, uint32_t r, uint32_t vix, const DJob& J,
                                  uint64_t fm, bool maybe, const uint8_t* v, uint32_t n) {
  for (uint32_t q = 0; q < J.jdfa_count; q++) {
    const DJobDfa jd = P.jdfas[J.jdfa_begin + q];
    uint64_t al = 0;
    for (uint64_t f = fm; f; f &= f - 1) al |= P.u64pool[jd.fmask_off + (__ffsll((unsigned long long)f) - 1)];
    if (!al) continue;
    uint64_t x = al;
    if (!maybe) x &= scan_full(P, P.dfas[jd.dfa], v, n) ^ jd.neg_mask;
    while (x) {
      const int k = __ffsll((unsigned long long)x) - 1;
      x &= x - 1;
      hit_value(B, P.pats[jd.pat_begin + k].slot, r, vix, maybe ? 1u : 0u);
    }
  }
}

// Patterns of automaton q the admitting filters fm let through (image table).
__device__ __forceinline__ uint64_t img_allowed(const uint8_t* img, uint32_t fmask_off, uint32_t nf, uint32_t q,
                                                uint64_t fm) {
  uint64_t a = 0;
  for (uint64_t f = fm; f; f &= f - 1)
    a |= *(const uint64_t*)(img + fmask_off + 8 * (q * nf + (__ffsll((unsigned long long)f) - 1)));
  return a;
}

// r: the queue lane's global item index
__device__ __forceinline__ void emit_img(const DBatch& B, uint32_t r, const uint8_t* img, uint32_t slots_off,
                                         uint64_t x) {
  while (x) {
    const int k = __ffsll((unsigned long long)x) - 1;
    x &= x - 1;
    hit_item(B, *(const uint32_t*)(img + slots_off + 4 * k), r);
  }
}

// Accepting transition of union automaton q (rare): emit its matches now.
__device__ void union_accept(const DProgram& P, const DBatch& B, uint32_t r, const DJob& J, const uint8_t* img,
                             uint32_t nf, uint32_t q, uint64_t fm, uint32_t st, uint32_t cls) {
  const DJobDfa jd = gi_cload(P.jdfas, J.jdfa_begin + q);
  const DDfa d = gi_cload(P.dfas, (uint64_t)jd.dfa);
  const uint64_t x = P.u64pool[d.acc_off + st * 5 + img[jd.lds_combo + cls]] & img_allowed(img, J.lds_fmask, nf, q, fm);
  if (x) emit_img(B, r, img, jd.lds_slots, x);
}

// End of a value: end-of-input matches of every automaton (negation applied).
// The value's hits are committed together: its item record and request layout
// are read once, its value-signature bits go out in one atomicOr, and the hit
// words of slots < 128 are ORed per word first (one atomic per touched word
// instead of one per hit).  The exact hit-set keys stay one per hit.
__device__ void value_end(const DProgram& P, const DBatch& B, uint32_t idx, const DJob& J, const uint8_t* img,
                          uint32_t nf, uint32_t K, uint64_t fm, const uint32_t* st) {
  uint32_t r = 0, vix = GI_NO_VIX, vbits = 0, hw0 = 0, hw1 = 0, hw2 = 0, hw3 = 0;
  bool any = false;
  ReqLayout L{};
  for (uint32_t q = 0; q < K; q++) {
    const DJobDfa jd = gi_cload(P.jdfas, J.jdfa_begin + q);
    GI_BOUND(st[q] < P.dfas[jd.dfa].n_states, st[q], q);
    const uint64_t al = img_allowed(img, J.lds_fmask, nf, q, fm);
    if (!al) continue;
    const DDfa d = gi_cload(P.dfas, (uint64_t)jd.dfa);
    uint64_t bits;
    if (d.multi) bits = *(const uint64_t*)(img + jd.lds_endacc + 8 * st[q]);
    else bits = img[jd.lds_endacc + st[q]] ? 1ull : 0ull;
    uint64_t x = (bits ^ jd.neg_mask) & al;
    if (x && !any) {
      any = true;
      GI_BOUND(idx < B.items_cap, idx, B.items_cap);
      const uint2 rm = *(const uint2*)((const uint8_t*)B.items + 32ull * idx + 24);  // (req, meta)
      r = rm.x;
      vix = meta_vix(rm.y);
      if (vix != GI_NO_VIX) L = B.layout[r];
    }
    while (x) {
      const int k = __ffsll((unsigned long long)x) - 1;
      x &= x - 1;
      const uint32_t slot = *(const uint32_t*)(img + jd.lds_slots + 4 * k);
      const uint32_t bit = 1u << (slot & 31);
      vbits |= bit;
      const uint32_t w = slot >> 5;
      hw0 |= w == 0 ? bit : 0u;
      hw1 |= w == 1 ? bit : 0u;
      hw2 |= w == 2 ? bit : 0u;
      hw3 |= w == 3 ? bit : 0u;
      if (w >= 4) set_hit(B, slot, r);
      if (vix != GI_NO_VIX && L.hset_mask) hset_insert(B, L, slot, vix, 0u);
    }
  }
  if (!any) return;
  if (hw0) atomicOr(&B.hits[r], hw0);
  if (hw1) atomicOr(&B.hits[(uint64_t)B.rstride + r], hw1);
  if (hw2) atomicOr(&B.hits[2ull * B.rstride + r], hw2);
  if (hw3) atomicOr(&B.hits[3ull * B.rstride + r], hw3);
  if (vix != GI_NO_VIX) {
    GI_BOUND(vix < L.vmap_bits, vix, L.vmap_bits);
    atomicOr(&B.vmap[L.vmap_bit + vix], vbits);  // the value's slot signature
  }
}

// One wave scans NB queue blocks (<= 64 values each, the job's stream) at
// once: each lane steps NB independent values, so NB transition chains
// overlap their LDS latency (the automata of one value are already stepped
// in lockstep).
template <uint32_t NB>
__device__ __forceinline__ void scan_qblocks(const DProgram& P, const DBatch& B, const DJob& J, const uint8_t* img,
                                             uint32_t K, const uint32_t* trn, const uint32_t* st0, uint32_t umask,
                                             uint32_t nf, const uint2* d, uint32_t mode) {
  const uint32_t lane = lane_id();
  uint32_t req[NB], len[NB], nwl[NB], nwmax = 0, p0[NB], p1[NB];
  uint64_t fm[NB];
  const uint32_t* wp[NB];
  uint32_t st[NB][GI_JOB_MAX_DFA];
#pragma unroll
  for (uint32_t j = 0; j < NB; j++) {
    const uint64_t woff = (uint64_t)d[j].x << 2;
    const uint32_t nv = d[j].y & 0xFFu, nw = (d[j].y >> 8) & GI_QB_NW_MASK;
    GI_BOUND(nv <= 64 && woff + (uint64_t)(GI_QB_HDR + nw) * nv <= B.pool_cap, d[j].x, d[j].y);
    const uint32_t* q = B.pool + woff;
    req[j] = 0;
    len[j] = 0;
    fm[j] = 0;
    bool act = false;
    if (lane < nv) {
      req[j] = q[lane];
      GI_BOUND(req[j] < B.items_cap, req[j], 0u);
      fm[j] = B.igm[req[j]];
      len[j] = q[nv + lane];
      GI_BOUND(req[j] < B.items_cap && len[j] <= 4 * nw, req[j], len[j]);  // req: global item index
      uint64_t any = 0;
      for (uint32_t k = 0; k < K; k++) any |= img_allowed(img, J.lds_fmask, nf, k, fm[j]);
      act = any != 0;
    }
    if (mode & 2) act = false;
    nwl[j] = (act && !(mode & 4)) ? (len[j] + 3) / 4 : 0u;
    if (!act) len[j] = 0xFFFFFFFFu;  // marks an idle lane (no value_end)
    nwmax = max(nwmax, nw);
    wp[j] = q + GI_QB_HDR * nv + lane;
    // this lane's words, loaded two ahead of the automaton steps
    p0[j] = nwl[j] > 0 ? wp[j][0] : 0u;
    p1[j] = nwl[j] > 1 ? wp[j][nv] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < GI_JOB_MAX_DFA; k++) st[j][k] = st0[k];
  }
  if (mode & 16) umask = 0;
  const uint32_t* jam = (const uint32_t*)img;
  for (uint32_t w = 0; w < nwmax; w++) {
    uint32_t wd[NB];
#pragma unroll
    for (uint32_t j = 0; j < NB; j++) {
      const uint32_t nv = d[j].y & 0xFFu;
      wd[j] = p0[j];
      p0[j] = p1[j];
      p1[j] = w + 2 < nwl[j] ? wp[j][(uint64_t)(w + 2) * nv] : 0u;
    }
#pragma unroll
    for (uint32_t b = 0; b < 4; b++) {
#pragma unroll
      for (uint32_t j = 0; j < NB; j++) {
        if (w < nwl[j] && 4 * w + b < len[j]) {
          const uint32_t jm = jam[(wd[j] >> (8 * b)) & 0xFFu];  // ASCII or GI_RUNE_MARK
#pragma unroll
          for (uint32_t q = 0; q < GI_JOB_MAX_DFA; q++) {
            if (q < K) {
              const uint32_t cls = (jm >> (8 * q)) & 0xFFu;
              const uint32_t tv = *(const uint16_t*)(img + (trn[q] & 0xFFFFFu) + 2 * (st[j][q] * (trn[q] >> 20) + cls));
              if ((umask >> q) & 1u) {
                if (tv & 0x8000u) union_accept(P, B, req[j], J, img, nf, q, fm[j], st[j][q], cls);
                st[j][q] = tv & 0x7FFFu;
              } else {
                st[j][q] = tv;
              }
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < NB; j++)
    if (len[j] != 0xFFFFFFFFu && !(mode & 8)) value_end(P, B, req[j], J, img, nf, K, fm[j], st[j]);
}

// Persistent kernel over units (job, 1024 queue-block entries), job-major.
// Each wave reads 64 entries of its job's stream list (one per lane) and scans
// the non-empty ones one after the other.  LDS: the job image is copied once
// per job change; !LDS: the image is read from HBM (automata too large for LDS).
// BIG: the 1-workgroup-per-CU launch of images above 64 KB (its own symbol,
// so per-kernel profiles keep the two launches apart).
#ifndef GI_SCAN_NB
// queue blocks a wave steps at once (independent LDS transition chains).
// Measured on C2 (1M): 1 block at 8 waves/SIMD, 62 VGPRs, no spills: 17.96 ms,
// WRITE_SIZE 1.37 GB; 2 blocks at 8 waves/SIMD (64 VGPRs, 27 spills, 112 B
// scratch/lane): 18.89 ms, 9.3 GB of spill writes; 2 at 6 waves: 22.6 ms.
#define GI_SCAN_NB 1
#endif
#ifndef GI_SCAN_WPE
#define GI_SCAN_WPE 8  // k_scan: 8 waves/SIMD; 6 (1 block: 21.9 ms) and 4 (2 blocks: 22.2 ms) are slower
#endif
template <bool LDS, bool BIG>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(GI_SCAN_WPE, 8))) k_scan(DProgram P, DBatch B, const uint32_t* __restrict__ jl, uint32_t n_jl,
                                               uint32_t mode, uint32_t acct_slot) {
  uint64_t rwords = 0;  // queue words of this launch's streams, each counted once (algorithmic bytes)
  uint64_t rsteps = 0;  // automaton byte-steps (padded words x 4 x automata of the job)
  extern __shared__ __attribute__((aligned(16))) uint8_t simg[];
  __shared__ uint2 clist[1024];
  __shared__ uint32_t wcnt[16];
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nwv = blockDim.x >> 6;
  const uint32_t n_iw = min(B.ibk[3 * GI_NB], B.qcap);
  const uint32_t per_unit = blockDim.x;  // entries per unit
  const uint32_t nu_job = (n_iw + per_unit - 1) / per_unit;
  // Unit order.  XCD-grouped (default): the jobs of one chunk of queue blocks
  // are consecutive units of one XCD (workgroup b runs on XCD b % 8 and the
  // grid is a multiple of 8), so the jobs of a stream -- adjacent in jl --
  // read that chunk's queue words while they are in the XCD's L2 instead of
  // each fetching them from HBM.  GI_SCAN_MODE bit 5 (32): job-major (each
  // job sweeps all chunks, the round-4 order).
  // (a job with fewer than 8 chunks -- few requests, e.g. C5's 32 -- would
  // leave the XCDs past its last chunk idle: job-major then)
  const uint32_t ngrp = (nu_job + 7) / 8;
  const bool xcd = !(mode & 32) && (gridDim.x & 7) == 0 && nu_job >= 8;
  const uint64_t n_units = xcd ? (uint64_t)ngrp * 8 * n_jl : (uint64_t)nu_job * n_jl;
  uint32_t loaded = 0xFFFFFFFFu;
  for (uint64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    uint32_t jj, chunk;
    if (xcd) {
      const uint64_t q = u >> 3;
      jj = (uint32_t)(q % n_jl);
      chunk = (uint32_t)(q / n_jl) * 8u + (uint32_t)(u & 7u);
      if (chunk >= nu_job) continue;  // (block-uniform)
    } else {
      jj = (uint32_t)(u / nu_job);
      chunk = (uint32_t)(u - (uint64_t)jj * nu_job);
    }
    const uint32_t j = jl[jj];
    const DJob J = gi_cload(P.jobs, j);
    const uint8_t* img = P.images + J.img_off;
    if (LDS) {
      if (j != loaded) {  // block-uniform
        __syncthreads();
        const uint4* src = (const uint4*)(P.images + J.img_off);
        for (uint32_t k = threadIdx.x; k < (J.img_bytes + 15) / 16; k += blockDim.x) ((uint4*)simg)[k] = src[k];
        __syncthreads();
        loaded = j;
      }
      img = simg;
    }
    if (mode & 1) continue;
    // compact the unit's non-empty queue blocks into LDS, then deal them out
    // to the 16 waves round-robin (balanced within the workgroup)
    const uint32_t e = chunk * per_unit + wv * 64 + lane;
    uint2 mine = make_uint2(0u, 0u);
    if (e < n_iw) mine = B.qblk[(uint64_t)J.stream * B.qcap + e];
    if (!stage_runs(B, (mine.y & GI_QB_BODY) != 0, J.prefix)) mine.y = 0;
    const uint64_t live = __ballot((mine.y & 0xFFu) != 0);
    if (lane == 0) wcnt[wv] = __popcll(live);
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (uint32_t w = 0; w < nwv; w++) {
      const uint32_t c = wcnt[w];
      wbase += w < wv ? c : 0u;
      total += c;
    }
    if ((mine.y & 0xFFu) != 0) clist[wbase + mask_rank(live)] = mine;
    __syncthreads();
    const uint32_t nf = P.n_gfilters;  // fmask tables are indexed by global filter id
    const uint32_t K = J.jdfa_count;
    uint32_t trn[GI_JOB_MAX_DFA], st0[GI_JOB_MAX_DFA], umask = 0;
#pragma unroll
    for (uint32_t k = 0; k < GI_JOB_MAX_DFA; k++) {
      trn[k] = 0;
      st0[k] = 0;
      if (k < K) {
        const DJobDfa jd = gi_cload(P.jdfas, J.jdfa_begin + k);
        const DDfa d = gi_cload(P.dfas, (uint64_t)jd.dfa);
        trn[k] = (uint32_t)jd.lds_trans | (d.n_classes << 20);
        st0[k] = d.start;
        if (d.multi) umask |= 1u << k;
      }
    }
    // jl is sorted by stream: only the first job of a stream counts its words
    const bool first = jj == 0 || gi_cload(P.jobs, jl[jj - 1]).stream != J.stream;
    for (uint32_t i = wv; i < total; i += GI_SCAN_NB * nwv) {  // GI_SCAN_NB blocks per wave at a time
      uint2 d[GI_SCAN_NB];
#pragma unroll
      for (uint32_t j = 0; j < GI_SCAN_NB; j++) d[j] = i + j * nwv < total ? clist[i + j * nwv] : make_uint2(0u, 0u);
#pragma unroll
      for (uint32_t j = 0; j < GI_SCAN_NB; j++) {
        const uint32_t dnw = (d[j].y >> 8) & GI_QB_NW_MASK;
        const uint64_t w = (uint64_t)(d[j].y & 0xFFu) * (GI_QB_HDR + dnw);
        rwords += (first && !(d[j].y & GI_QB_SHARED)) ? w : 0;  // a shared block is counted at its writer
        rsteps += (uint64_t)(d[j].y & 0xFFu) * dnw * 4 * K;
      }
      scan_qblocks<GI_SCAN_NB>(P, B, J, img, K, trn, st0, umask, nf, d, mode);
    }
    __syncthreads();  // clist / wcnt reuse
  }
  if ((threadIdx.x & 63) == 0 && rwords) atomicAdd(&B.acct[10 + acct_slot], (unsigned long long)rwords);
  if ((threadIdx.x & 63) == 0 && rsteps) atomicAdd(&B.acct[13 + acct_slot], (unsigned long long)rsteps);

}

// REQUEST_BODY targets of phase-2 links (residual: the variable only exists
// after ProcessRequestBody), tested on the speculative body of k_collect.
// k_eval relies on these bits only when phase 1 ended with k_collect's
// processor (REQUEST_BODY is then exactly the body).
//
// One wave per body (the batch's body list, longest first).  The links come
// ordered by transformation chain (compile.cpp); each chain runs once per body
// and every link's operator is evaluated on its output, both split over the 64
// lanes at "sync points" -- positions where the sequential algorithm is
// provably in its initial state whatever came before:
//   * a transformation stage: lane L runs the unchanged sequential
//     transformation over [s_L, s_L+1) (s_L = the first sync point at or after
//     L/64 of the input), writing to a 3x-scaled slot of the other buffer; a
//     wave prefix sum of the output lengths then packs the chunks.  The
//     concatenation equals the whole-input result because no escape sequence
//     straddles a sync point and each chunk starts in the initial state;
//   * an automaton: lane L steps its chunk from the state reached after a
//     64-byte warm-up ending at s_L (started in the start state); lane L's
//     result is exact iff its warm state equals lane L-1's exact final state
//     (a DFA state fixes the whole future), which the wave checks lane by lane,
//     rescanning a chunk from the exact state where it is not (rare: a pattern
//     that remembers more than 64 bytes, e.g. "a.*b");
//   * @validate*: each chunk evaluated independently (byte-local checks).
// Transformations without sync points (trim, normalizePath, base64Decode,
// digests, ...) and operators without an automaton run on lane 0 alone.
// A chain overflow sets the chain's link bits ("maybe": k_eval evaluates).

// true: transformation `code` can be split at sync points (t_sync)
__device__ __forceinline__ bool t_chunkable(uint8_t code) {
  switch (code) {
    case T_LOWERCASE: case T_UTF8TOUNICODE: case T_REMOVENULLS: case T_REPLACENULLS: case T_REMOVEWHITESPACE:
    case T_URLENCODE: case T_HEXENCODE: case T_BASE64ENCODE: case T_COMPRESSWHITESPACE: case T_CMDLINE:
    case T_URLDECODE: case T_URLDECODEUNI: case T_JSDECODE: case T_CSSDECODE: case T_HTMLENTITYDECODE:
      return true;
  }
  return false;
}

__device__ __forceinline__ bool no_byte_before(const uint8_t* s, uint32_t p, uint32_t w, uint8_t c) {
  for (uint32_t k = 1; k <= w && k <= p; k++)
    if (s[p - k] == c) return false;
  return true;
}

// Is position p (0 < p < n) of s a sync point of transformation `code`?
// (the sequential state at p is initial, and no escape sequence starting
// before p reads s[p]: see the transformation's code above)
__device__ __forceinline__ bool t_sync(uint8_t code, const uint8_t* s, uint32_t p) {
  const uint8_t c = s[p - 1];
  switch (code) {
    case T_LOWERCASE: case T_UTF8TOUNICODE: return s[p] < 0x80;  // a rune start (ASCII never continues one)
    case T_REMOVENULLS: case T_REPLACENULLS: case T_REMOVEWHITESPACE: case T_URLENCODE: case T_HEXENCODE:
      return true;
    case T_BASE64ENCODE: return p % 3 == 0;
    case T_COMPRESSWHITESPACE: return !ws_or_nbsp(c);
    case T_CMDLINE:  // a kept character resets the pending-space state
      return !(c == '"' || c == '\'' || c == '\\' || c == '^' || c == ' ' || c == ',' || c == ';' || c == '\t' ||
               c == '\r' || c == '\n');
    case T_URLDECODE: return no_byte_before(s, p, 2, '%');
    case T_URLDECODEUNI: return no_byte_before(s, p, 5, '%');   // %uXXXX
    case T_JSDECODE: return no_byte_before(s, p, 5, '\\');      // \uXXXX
    case T_CSSDECODE: return no_byte_before(s, p, 7, '\\');     // \ + 6 hex + 1 space
    case T_HTMLENTITYDECODE:  // an entity never contains '&', and ends at the first byte outside [#0-9A-Za-z]
      return s[p] == '&' || !(isalnum_(c) || c == '#' || c == '&');
  }
  return false;
}

// lane's chunk [*a, *e) of s[0, n): sync points found per lane from L/64 of
// the input (sync(p) decides); a lane without one inside its nominal range
// gets an empty chunk and the previous lane runs through.
template <class F>
__device__ __forceinline__ void wave_chunks(uint32_t n, F&& sync, uint32_t* a, uint32_t* e) {
  const uint32_t L = lane_id();
  const uint32_t a0 = (uint32_t)((uint64_t)n * L / 64), a1 = (uint32_t)((uint64_t)n * (L + 1) / 64);
  uint32_t sp = L == 0 ? 0u : 0xFFFFFFFFu;
  for (uint32_t p = max(a0, 1u); L > 0 && p < a1 && sp == 0xFFFFFFFFu; p++)
    if (sync(p)) sp = p;
  const uint64_t valid = __ballot(sp != 0xFFFFFFFFu);
  const uint64_t after = L == 63 ? 0ull : valid & (~0ull << (L + 1));
  const uint32_t nxt = after ? (uint32_t)(__ffsll((unsigned long long)after) - 1) : 64u;
  const uint32_t ne = __shfl(sp, nxt == 64 ? 0 : (int)nxt, 64);
  *a = sp;
  *e = sp == 0xFFFFFFFFu ? sp : (nxt == 64 ? n : ne);
}


// single (sticky) automaton d over s[from, to) of s[0, n) from state st;
// returns the state (d.accept once a match completed).  tr / amap: the
// transition table and ASCII class map (LDS copies when they fit); the text
// is read a word at a time.
__device__ __forceinline__ uint32_t dfa_steps(const DProgram& P, const DDfa& d, const uint16_t* __restrict__ tr,
                                              const uint8_t* __restrict__ amap, const uint8_t* s, uint32_t n,
                                              uint32_t from, uint32_t to, uint32_t st) {
  const uint32_t ncls = d.n_classes;
  uint32_t i = from;
  uint32_t win = 0, wbeg = 0, wend = 0;
  while (i < to && st != d.accept) {
    if (i >= wend) {
      win = load_u32u(s + i);
      wbeg = i;
      wend = i + 4;
    }
    const uint8_t c = (uint8_t)(win >> (8 * (i - wbeg)));
    uint32_t cls;
    if (d.byte_mode || c < 0x80) {
      cls = amap[c];
      i++;
    } else {
      uint32_t w;
      const uint32_t r = decode_rune(s, n, i, &w);
      i += w;
      cls = rune_class(P, d, r);
    }
    st = tr[st * ncls + cls];
  }
  return st;
}

// k_body's operators other than automata / @validate*, on lane 0 (rare: the
// compiler keeps detectors out of k_body).  Out of line, so the interpreter
// state it needs stays out of k_body's register budget.
__device__ __noinline__ bool body_other_op(const DProgram& P, const Region& g, const DOp& o, const uint8_t* s,
                                           uint32_t n) {
  Tx t;
  t.P = &P;
  t.t0 = g.t0;
  t.t1 = g.t1;
  t.cap_t = g.cap_t;
  t.mt = g.mt;
  t.cap_mt = g.cap_mt;
  t.flags = 0;
  return eval_op<false>(t, o, s, n);
}

#define GI_BODY_LDS 16384  // k_body's LDS automaton slot (bytes): 8 one-wave workgroups per CU

// Exact "d matches somewhere in s[0, n)" by the whole wave (see above).
// lds: GI_BODY_LDS bytes of the workgroup's LDS for the automaton tables.
__device__ bool wave_dfa_match(const DProgram& P, const DDfa& d, const uint8_t* s, uint32_t n, uint8_t* lds) {
  const uint32_t L = lane_id();
  const uint32_t tb = d.n_states * d.n_classes * 2, ab = d.byte_mode ? 256u : 128u;
  const bool in_lds = tb + ab <= GI_BODY_LDS;
  const uint16_t* tr = P.trans + d.trans_off;
  const uint8_t* amap = P.u8pool + d.amap_off;
  if (in_lds) {
    __syncthreads();  // the previous link's tables are no longer read
    for (uint32_t k = L; k < tb / 2; k += 64) ((uint16_t*)lds)[k] = tr[k];
    for (uint32_t k = L; k < ab; k += 64) lds[tb + k] = amap[k];
    __syncthreads();
    tr = (const uint16_t*)lds;
    amap = lds + tb;
  }
  uint32_t a, e;
  if (d.byte_mode) wave_chunks(n, [&](uint32_t) { return true; }, &a, &e);
  else wave_chunks(n, [&](uint32_t p) { return s[p] < 0x80; }, &a, &e);
  const bool act = a != 0xFFFFFFFFu;
  uint32_t warm = d.start, fin = d.start;
  if (act && a > 0) {
    uint32_t w = a > 64 ? a - 64 : 0u;
    if (!d.byte_mode)
      while (w < a && s[w] >= 0x80) w++;  // a rune start (s[a] is ASCII)
    warm = dfa_steps(P, d, tr, amap, s, n, w, a, d.start);
    if (warm == d.accept) warm = 0xFFFFFFFFu;  // a warm-up match proves nothing: no guess
  }
  if (act && warm != 0xFFFFFFFFu) fin = dfa_steps(P, d, tr, amap, s, n, a, e, warm);
  const uint64_t actm = __ballot(act);
  // lane by lane: exact state entering each chunk
  uint32_t ex = d.start;
  for (uint64_t m = actm; m; m &= m - 1) {
    const int k = __ffsll((unsigned long long)m) - 1;
    const uint32_t gk = __shfl(warm, k, 64), fk = __shfl(fin, k, 64);
    const uint32_t ak = __shfl(a, k, 64), ek = __shfl(e, k, 64);
    if (gk == ex) {
      ex = fk;
    } else {  // mispredicted: rescan the chunk from the exact state (lane 0)
      uint32_t x = 0;
      if (L == 0) x = dfa_steps(P, d, tr, amap, s, n, ak, ek, ex);
      ex = __shfl(x, 0, 64);
    }
    if (ex == d.accept) return true;
  }
  return P.u8pool[d.endacc_off + ex] != 0;
}

// @validate* over s[0, n) by the whole wave: chunk results OR-ed
__device__ bool wave_validate(const DOp& o, const uint8_t* s, uint32_t n) {
  if (o.kind == OP_UNCONDITIONAL) return true;
  uint32_t a, e;
  if (o.kind == OP_VALIDATE_BYTE_RANGE) wave_chunks(n, [&](uint32_t) { return true; }, &a, &e);
  else if (o.kind == OP_VALIDATE_URL_ENCODING) wave_chunks(n, [&](uint32_t p) { return no_byte_before(s, p, 2, '%'); }, &a, &e);
  else wave_chunks(n, [&](uint32_t p) { return s[p] < 0x80; }, &a, &e);
  bool r = false;
  if (a != 0xFFFFFFFFu && e > a) r = validate_op(o.kind, o.bits, s + a, e - a);
  return __ballot(r) != 0;
}

// Chunkable transformation `code` of src[0, n) into dst (cap bytes, never
// src) by the whole wave, through LDS tiles of GI_TT_IN input bytes: the tile
// is read coalesced into LDS, each lane transforms the chunk between its sync
// points (t_sync) LDS -> LDS, and the compacted output is written coalesced.
// A lane streaming its own chunk straight from HBM touches one cache line per
// lane per byte, and 64 lanes x 8+ waves of such streams thrash the CU's L1
// (k_body spent ~1.6 ms per 23 KB body on a 3-transform chain that way).
// A tile that is not the last ends at the last lane's sync point (that
// lane's chunk starts the next tile), so every chunk lies between two sync
// points exactly as in the one-shot split; sync points are tested on
// tile-relative positions, which is exact because the tile start is itself
// a sync point of the same rule (no escape byte within the look-back window
// before it; base64Encode's p % 3 holds since the start is 0 mod 3).  A tile
// without an inner sync point is done by lane 0 from HBM up to the next one.
// Returns the output length, -1 on overflow; *psumm = byte summary of it.
#define GI_TT_IN 3072
#define GI_TT_LDS (GI_TT_IN + 32 + 3 * GI_TT_IN + 8 * 64 + 2 * 65 * 4)
static_assert(GI_TT_LDS <= 16384, "k_body's LDS slot holds the transformation tiles");
__device__ __forceinline__ int64_t wave_transform_lds(const DProgram& P, uint8_t code, const uint8_t* src, uint32_t n, uint8_t* dst,
                                      uint64_t cap, uint8_t* lds, uint32_t* psumm) {
  const uint32_t L = lane_id();
  uint8_t* const inb = lds;                // the tile's 16-byte words (GI_TT_IN + 32 bytes)
  uint8_t* out = lds + GI_TT_IN + 32;  // lane slots at 3 * a + 8 * L (3x + 8 bytes each, as apply_transform allows)
  uint32_t* offs = (uint32_t*)(out + 3 * GI_TT_IN + 8 * 64);  // [65] output offsets
  uint32_t* slot = offs + 65;                                  // [64] slot starts
  uint64_t o = 0;
  uint32_t summ = 0;
  uint32_t base = 0;
  while (base < n) {
    const uint32_t tn = min(n - base, (uint32_t)GI_TT_IN);
    const bool last = base + tn == n;
    __syncthreads();  // the previous tile's LDS reads are done
    // the tile as aligned 16-byte words, all loads in flight at once (the
    // sources -- the body arena, the request's 16-byte aligned t0 / t1 --
    // are readable 15 bytes either side)
    const uintptr_t a0 = (uintptr_t)(src + base);
    const uint32_t sh = (uint32_t)(a0 & 15u);
    const uint4* w = (const uint4*)(a0 - sh);
    for (uint32_t k = L; k < (sh + tn + 15) / 16; k += 64) ((uint4*)inb)[k] = w[k];
    const uint8_t* in = inb + sh;
    __syncthreads();
    uint32_t a, e;
    wave_chunks(tn, [&](uint32_t p) { return t_sync(code, in, p); }, &a, &e);
    bool act = a != 0xFFFFFFFFu && e > a;
    uint32_t adv = tn;
    if (!last) {  // the last lane with a sync point carries its chunk to the next tile
      const uint64_t v = __ballot(a != 0xFFFFFFFFu);
      const int hi = 63 - __builtin_clzll((unsigned long long)v);
      if (hi == 0) {  // no sync point inside the tile: lane 0 runs to the next one, from HBM
        int64_t m = 0;
        uint32_t sm = 0, stop = n;
        if (L == 0) {
          for (uint32_t p = base + tn; p < n; p++)
            if (t_sync(code, src + base, p - base)) {
              stop = p;
              break;
            }
          m = apply_transform(P, code, src + base, stop - base, dst + o, (uint32_t)min(cap - o, (uint64_t)0xFFFFFFFFu));
          if (m > 0) sm = value_summary(dst + o, (uint32_t)m);
        }
        m = __shfl(m, 0, 64);
        if (m < 0) return -1;
        summ |= sm;
        o += (uint64_t)m;
        base = __shfl(stop, 0, 64);
        continue;
      }
      adv = __shfl(a, hi, 64);
      if ((int)L == hi) act = false;
    }
    // (the tile pointers as LDS pointers: the transformation's accesses are ds_* ops)
    int64_t m = act ? apply_transform_tile(P, code, (const gi_lds_u8*)(in + a), e - a,
                                           (gi_lds_u8*)(out + 3u * a + 8u * L), 3 * (e - a) + 8)
                    : 0;
    if (__ballot(m < 0) != 0) return -1;
    uint32_t tot = 0;
    const uint32_t o0 = wave_excl_sum((uint32_t)m, &tot);
    if (o + tot > cap) return -1;
    const uint32_t st = act ? 3u * a + 8u * L : 0u;
    for (uint32_t i = 0; i < (uint32_t)max(m, (int64_t)0); i++) summ |= byte_summary(out[st + i]);
    offs[L] = o0;
    slot[L] = st;
    if (L == 0) offs[64] = tot;
    __syncthreads();
    uint32_t k = 0;
    for (uint32_t j = L; j < tot; j += 64) {
      while (k < 63 && offs[k + 1] <= j) k++;
      dst[o + j] = out[slot[k] + (j - offs[k])];
    }
    o += tot;
    base += adv;
  }
  for (int x = 32; x > 0; x >>= 1) summ |= (uint32_t)__shfl_xor((int)summ, x, 64);
  *psumm = summ;
  return (int64_t)o;
}

// One wave runs transformation chain (off, len) over v[0, *cn): chunk-parallel
// for the chunkable transformations (t_sync boundaries), lane 0 otherwise.
// t0 / t1 are the two cap-byte buffers; *cur / *cn are the input on entry
// and the output on return; false on overflow.  summ = byte summary of v.
// tiles: the chunkable ones run LDS-tiled in lds (GI_TT_LDS bytes of the
// workgroup's LDS; inlined, so every tile access is a ds_* op -- a generic
// pointer would let the compiler merge byte stores into misaligned wider
// flat stores, which fault on an LDS address).
__device__ __forceinline__ bool wave_run_chain(const DProgram& P, uint32_t off, uint32_t len, const uint8_t* src0, uint8_t* t0,
                               uint8_t* t1, uint64_t cap, uint32_t summ, const uint8_t** pcur, uint32_t* pcn,
                               uint8_t* lds = nullptr, bool tiles = false) {
  const uint32_t L = threadIdx.x;
  const uint8_t* cur = *pcur;
  uint32_t cn = *pcn;
  bool ok = true;
  for (uint32_t q = 0; q < len && ok; q++) {
    const uint8_t code = (uint8_t)P.tchains[off + q];
    if (transform_identity(summ, code)) continue;
    if (tiles && t_chunkable(code)) {
      uint8_t* dst = cur == t0 ? t1 : t0;
      uint32_t sm = 0;
      const int64_t m = wave_transform_lds(P, code, cur, cn, dst, cap, lds, &sm);
      if (m < 0) {
        ok = false;
      } else {
        cur = dst;
        cn = (uint32_t)m;
        summ = sm;
      }
      continue;
    }
    // buffers: tmp / dst are the two transformation buffers other than cur
    uint8_t* tmp = cur == t1 ? t0 : t1;
    uint8_t* dst = cur == src0 ? t0 : (uint8_t*)cur;
    if (dst == tmp) dst = tmp == t0 ? t1 : t0;
    int64_t outn = -1;
    if (t_chunkable(code) && 3ull * cn + 8 * 64 <= cap) {
      const uint8_t* src = cur;
      uint32_t a, e;
      wave_chunks(cn, [&](uint32_t p) { return t_sync(code, src, p); }, &a, &e);
      const bool act = a != 0xFFFFFFFFu && e > a;
      uint8_t* lt = tmp + 3ull * (act ? a : 0u) + 8u * L;
      int64_t m = act ? apply_transform_inl(P, code, src + a, e - a, lt, 3 * (e - a) + 8) : 0;
      uint32_t tot = 0, o0 = 0;
      if (__ballot(m < 0) == 0) o0 = wave_excl_sum((uint32_t)m, &tot);
      const bool bad = __ballot(m < 0) != 0 || tot > cap;
      if (!bad) {
        __syncthreads();  // tmp written; dst (possibly the source) is free
        uint32_t sm = m > 0 ? value_summary(lt, (uint32_t)m) : 0u;
        copy_bytes(dst + o0, lt, (uint32_t)max(m, (int64_t)0));
        for (int x = 32; x > 0; x >>= 1) sm |= (uint32_t)__shfl_xor((int)sm, x, 64);
        summ = sm;
        __syncthreads();
        outn = tot;
        cur = dst;
      }
    } else {  // sequential on lane 0
      int m = 0;
      if (L == 0) m = (int)max(apply_transform(P, code, cur, cn, tmp, (uint32_t)min(cap, (uint64_t)0xFFFFFFFFu)), (int64_t)-1);
      m = __shfl(m, 0, 64);
      __syncthreads();
      if (m >= 0) {
        outn = m;
        cur = tmp;
        uint32_t a, e;
        wave_chunks((uint32_t)m, [&](uint32_t) { return true; }, &a, &e);
        uint32_t sm = (a != 0xFFFFFFFFu && e > a) ? value_summary(cur + a, e - a) : 0u;
        for (int x = 32; x > 0; x >>= 1) sm |= (uint32_t)__shfl_xor((int)sm, x, 64);
        summ = sm;
      }
    }
    if (outn < 0) ok = false;
    else cn = (uint32_t)outn;
  }
  *pcur = cur;
  *pcn = cn;
  return ok;
}

// Two waves per SIMD (the inlined LDS tile path would otherwise take the
// whole register file: 1 wave, k_body 68 -> 83 ms on C3 at 50k; with the cap,
// 17 spilled VGPRs and 46 ms).
#ifndef GI_BODY_WPE
#define GI_BODY_WPE 3  // C3 A/B: 3 waves/SIMD (168 VGPRs, 84 spilled) 164 ms, 2 waves (256 VGPRs) 174 ms
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GI_BODY_WPE, 8))) k_body(DProgram P, DBatch B) {
  __shared__ __attribute__((aligned(16))) uint8_t kb_lds[GI_BODY_LDS];
  const uint32_t L = threadIdx.x;
  for (uint32_t bi = blockIdx.x; bi < B.n_body; bi += gridDim.x) {
    const uint32_t r = B.body_list[bi];
    GI_BOUND(r < B.n_req, r, bi);
    if (B.stage == 2 && !B.pend[r]) continue;  // decided in phase 1
    const ReqHdr* H = (const ReqHdr*)(B.scratch + B.layout[r].base);
    if (H->spec_proc == BP_NONE || (H->flags & GI_REQ_ERROR_MASK)) continue;
    const Region g = region_of(P, B, r);
    gi_span bs = B.reqs[r].body;
    if (H->spec_proc == BP_MULTIPART) bs.len = 0;  // coraza's multipart processor sets no REQUEST_BODY
    const uint8_t* body = B.data + bs.off;
    const uint8_t* cur = body;
    uint32_t cn = bs.len;
    bool ok = true;
    uint32_t prev_off = 0xFFFFFFFFu, prev_len = 0;
    for (uint32_t k = 0; k < P.n_body_links; k++) {
      const DRule R = gi_cload(P.rules, (uint64_t)P.body_links[k]);
      // the gate: the first stage runs the links of the phase-2 prefix (its
      // k_eval stops before any other), the body stage the rest, for the
      // pending requests only
      if (B.stage && (B.stage == 1) != ((R.flags2 & RF2_PREFIX) != 0)) continue;
      const DOp o = gi_cload(P.ops, (uint64_t)R.op);
      const uint64_t c0 = B.prof ? gi_clock() : 0;
      bool same = R.tchain_len == prev_len;
      for (uint32_t q = 0; same && q < R.tchain_len; q++)
        same = P.tchains[R.tchain_off + q] == P.tchains[prev_off + q];
      if (!same) {  // run this link's chain over the body
        prev_off = R.tchain_off;
        prev_len = R.tchain_len;
        cur = body;
        cn = bs.len;
        ok = true;
        uint32_t summ = 0;
        {
          uint32_t a, e;
          wave_chunks(cn, [&](uint32_t) { return true; }, &a, &e);
          uint32_t m = (a != 0xFFFFFFFFu && e > a) ? value_summary(cur + a, e - a) : 0u;
          for (int q = 32; q > 0; q >>= 1) m |= (uint32_t)__shfl_xor((int)m, q, 64);
          summ = m;
        }
        ok = wave_run_chain(P, R.tchain_off, R.tchain_len, body, g.t0, g.t1, g.cap_t, summ, &cur, &cn, kb_lds, B.body_tiles != 0);
      }
      const uint64_t c1 = B.prof ? gi_clock() : 0;
      bool hit;
      if (!ok) {
        hit = true;  // chain overflow: maybe
      } else if ((o.kind == OP_RX || o.kind == OP_PM || (o.kind == OP_CONTAINS && o.arg_is_lit)) && o.nfa < 0 &&
                 o.dfa >= 0 && !P.dfas[o.dfa].multi) {
        bool m = false;
        for (uint32_t g = 0; g < max(o.ngroups, 1u) && !m; g++) m = wave_dfa_match(P, P.dfas[o.dfa + (int32_t)g], cur, cn, kb_lds);
        hit = m != (o.negate != 0);
      } else if (o.kind == OP_VALIDATE_BYTE_RANGE || o.kind == OP_VALIDATE_URL_ENCODING || o.kind == OP_VALIDATE_UTF8) {
        hit = wave_validate(o, cur, cn) != (o.negate != 0);
      } else {  // any other operator: lane 0, side-effect free
        bool h = false;
        if (L == 0) h = body_other_op(P, g, o, cur, cn);
        hit = __shfl((int)h, 0, 64) != 0;
      }
      if (hit && L == 0) set_hit(B, (uint32_t)R.hit_slot, r);
      if (B.prof && k < 16 && L == 0) {  // GI_PROF: cycles per link (transform, operator), per body
        gi_prof_add(&B.prof[96 + 2 * k], (unsigned long long)(c1 - c0));
        gi_prof_add(&B.prof[97 + 2 * k], (unsigned long long)(gi_clock() - c1));
      }
    }
  }
}

// Long values (>= GI_LONG_MIN bytes): one wave per (item, stream) listed by
// k_stream.  The stream's chain runs chunk-parallel (wave_run_chain) into the
// workgroup's two HBM buffers; the stream's automata are spread over the 64
// lanes, each a sequential full scan (no speculative chunk states to
// mispredict on 1 MB values), the validate operators run chunk-parallel and
// the detectors on lane 0 -> hit bits + value map.  An overflowing chain sets
// every admitted bit ("maybe", exact).
__global__ void __launch_bounds__(64) k_long(DProgram P, DBatch B) {
  __shared__ LiSqli lst;
  const uint32_t L = threadIdx.x;
  const uint32_t n = min(*B.long_count, B.long_cap);
  uint8_t* t0 = B.long_buf + (uint64_t)blockIdx.x * 2ull * B.long_bufcap;
  uint8_t* t1 = t0 + B.long_bufcap;
  for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {
    const uint2 ent = B.long_list[e];
    GI_BOUND(ent.x < B.items_cap && ent.y < P.n_streams, ent.x, ent.y);
    const Item it = ((const Item*)B.items)[ent.x];
    const DStream S = P.streams[ent.y];
    const uint64_t fm = B.igm[ent.x] & S.gmask;
    const uint32_t r = it.req, vix = meta_vix(it.meta);
    const uint32_t ik = item_kind(it);
    const bool body = ik == FK_ARG_POST || (ik >= FK_FILE && ik <= FK_FILE_SIZE);
    uint32_t summ;
    {
      uint32_t a, b;
      wave_chunks(it.vn, [&](uint32_t) { return true; }, &a, &b);
      uint32_t m = (a != 0xFFFFFFFFu && b > a) ? value_summary(it.vp + a, b - a) : 0u;
      for (int q = 32; q > 0; q >>= 1) m |= (uint32_t)__shfl_xor((int)m, q, 64);
      summ = m;
    }
    const uint8_t* cur = it.vp;
    uint32_t cn = it.vn;
    const bool ok = wave_run_chain(P, S.tchain_off, S.tchain_len, it.vp, t0, t1, B.long_bufcap, summ, &cur, &cn);
    // validate / detect operators of the stream
    for (uint32_t q = 0; q < S.val_count; q++) {
      const DScanVal sv = P.svals[S.val_begin + q];
      if (!(fm & sv.fmask) || !stage_runs(B, body, sv.prefix)) continue;
      bool hit = true;
      if (ok) {
        bool res;
        if (sv.kind == OP_DETECT_SQLI || sv.kind == OP_DETECT_XSS) {
          int x = 0;
          if (L == 0)
            x = sv.kind == OP_DETECT_SQLI ? li_detect_sqli(cur, cn, &lst, li_tables_const()) : li_detect_xss(cur, cn);
          res = __shfl(x, 0, 64) != 0;
        } else {
          DOp vo{};
          vo.kind = sv.kind;
          for (int k = 0; k < 8; k++) vo.bits[k] = sv.bits[k];
          res = wave_validate(vo, cur, cn);
        }
        hit = res != (sv.negate != 0);
      }
      if (hit && L == 0) hit_value(B, sv.slot, r, vix, ok ? 0u : 1u);
    }
    // automaton patterns: the stream's (job, automaton) pairs spread over the
    // lanes, each scanned sequentially over the whole value on the global
    // tables (scan_full: the union automaton's match mask, as k_scan_slow)
    uint32_t pair = 0;
    for (uint32_t j = 0; j < S.job_count; j++) {
      const DJob J = P.jobs[S.job_begin + j];
      if (!stage_runs(B, body, J.prefix)) continue;
      for (uint32_t q = 0; q < J.jdfa_count; q++, pair++) {
        if ((pair & 63u) != L) continue;
        const DJobDfa jd = P.jdfas[J.jdfa_begin + q];
        uint64_t al = 0;
        for (uint64_t f = fm; f; f &= f - 1) al |= P.u64pool[jd.fmask_off + (__ffsll((unsigned long long)f) - 1)];
        if (!al) continue;
        uint64_t x = al;
        if (ok) x &= scan_full(P, P.dfas[jd.dfa], cur, cn) ^ jd.neg_mask;
        while (x) {
          const int k = __ffsll((unsigned long long)x) - 1;
          x &= x - 1;
          hit_value(B, P.pats[jd.pat_begin + k].slot, r, vix, ok ? 0u : 1u);
        }
      }
    }
  }
}

// @detectSQLi / @detectXSS candidates, one lane per entry: libinjection with
// the tokenizer state in LDS; each detector runs at most once per entry and
// its result serves every admitting val of the masked streams.
// k_detect's cross-request memo of detector results (DBatch.dmemo_*): the
// detectors are pure functions of the value's bytes, and many candidates
// repeat across the requests of a batch (the same User-Agent or Referer
// string).  A thread claims an empty slot for its value's 64-bit hash, records
// where the value's bytes are (its det_bytes copy) and publishes each result
// as it computes it; a thread that finds the hash reuses a published result
// only after comparing the bytes with that copy (exact, whatever the hash),
// and otherwise computes the value itself.  Nobody waits on anybody.
#define GI_DM_VALID 1u
#define GI_DM_SQ_KNOWN 2u
#define GI_DM_SQ 4u
#define GI_DM_XS_KNOWN 8u
#define GI_DM_XS 16u
#define GI_DM_PROBES 16
__device__ __forceinline__ unsigned long long dm_hash(const uint8_t* v, uint32_t n) {
  unsigned long long h = 1469598103934665603ull ^ n;
  for (uint32_t i = 0; i < n; i++) h = (h ^ v[i]) * 1099511628211ull;
  return h | 1ull;  // never 0 (the empty key)
}
__device__ __forceinline__ bool dm_same(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (a[i] != b[i]) return false;
  return true;
}
// Results of the detectors the entry needs (bit 0 SQLi, bit 1 XSS).
__device__ uint32_t det_results(const DBatch& B, const uint8_t* v, uint32_t n, uint64_t off, bool need_s, bool need_x,
                                lid::LiSqli* st, const lid::LiTables& T, uint64_t* dsteps) {
  auto compute = [&](bool s) -> bool {
    if (!lid::li_candidate(s, v, n)) return false;
    *dsteps += n;
    return s ? lid::li_detect_sqli(v, n, st, T) : lid::li_detect_xss(v, n);
  };
  uint32_t out = 0;
  if (!B.dmemo_keys || n < B.dmemo_min) {  // (a short unique value costs more in memo round trips than to detect)
    if (need_s && compute(true)) out |= 1u;
    if (need_x && compute(false)) out |= 2u;
    return out;
  }
  const unsigned long long h = dm_hash(v, n);
  int32_t slot = -1;
  uint32_t state = 0;
  for (uint32_t p = 0; p < GI_DM_PROBES; p++) {
    const uint32_t i = (uint32_t)(h + p) & B.dmemo_mask;
    unsigned long long k = __atomic_load_n(&B.dmemo_keys[i], __ATOMIC_RELAXED);
    if (k == 0) {
      k = atomicCAS(&B.dmemo_keys[i], 0ull, h);
      if (k == 0) {  // claimed: record the canonical copy, then the results as they come
        B.dmemo_info[i] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), n, 0u);
        __threadfence();
        atomicOr(&B.dmemo_info[i].w, GI_DM_VALID);
        slot = (int32_t)i;
        state = GI_DM_VALID;
        break;
      }
    }
    if (k == h) {
      const uint32_t w = __atomic_load_n(&B.dmemo_info[i].w, __ATOMIC_ACQUIRE);
      if (w & GI_DM_VALID) {
        const uint4 inf = B.dmemo_info[i];
        const uint64_t coff = (uint64_t)inf.x | ((uint64_t)inf.y << 32);
        if (inf.z == n && coff + n <= B.det_bytes_cap && dm_same(v, B.det_bytes + coff, n)) {
          slot = (int32_t)i;
          state = w;
        }
      }
      break;  // (another value with this hash, or not published yet: compute alone)
    }
  }
  uint32_t pub = 0;
  if (need_s) {
    bool r;
    if (state & GI_DM_SQ_KNOWN) {
      r = (state & GI_DM_SQ) != 0;
    } else {
      r = compute(true);
      pub |= GI_DM_SQ_KNOWN | (r ? GI_DM_SQ : 0u);
    }
    out |= r ? 1u : 0u;
  }
  if (need_x) {
    bool r;
    if (state & GI_DM_XS_KNOWN) {
      r = (state & GI_DM_XS) != 0;
    } else {
      r = compute(false);
      pub |= GI_DM_XS_KNOWN | (r ? GI_DM_XS : 0u);
    }
    out |= r ? 2u : 0u;
  }
  if (slot >= 0 && pub) atomicOr(&B.dmemo_info[slot].w, pub);
  return out;
}

#ifndef GI_DETECT_LVAL
#define GI_DETECT_LVAL 0  // 1: short candidates staged in LDS (66 KB per workgroup: 2 workgroups per CU)
#endif
#ifndef GI_DETECT_WPE
#define GI_DETECT_WPE 3   // minimum waves per SIMD k_detect is compiled for.  Round 6, C2 A/B on one box: LVAL 0 +
                          // 3 waves (166 VGPRs, 48.3 KB LDS: 3 workgroups per CU) 10.9 ms, LVAL 1 + 1 wave (248
                          // VGPRs, 2 workgroups per CU) 12.9 ms; C3 198 vs 210 ms (make ab-det1 builds the latter)
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GI_DETECT_WPE))) k_detect(DProgram P,
                                                                                                   DBatch B) {
  __shared__ lid::LiSqli st[256];
#if GI_DETECT_LVAL
  // short candidates (<= 64 B, most of them) are read from LDS: stride 68 B =
  // 17 dwords per lane, conflict-free
  __shared__ __attribute__((aligned(16))) uint32_t lval[256 * 17];
#endif
  for (uint32_t i = threadIdx.x; i < LI_NWORDS; i += blockDim.x) lid::li_lw[i] = kLiWords[i];
  for (uint32_t i = threadIdx.x; i < LI_HASH_SIZE; i += blockDim.x) lid::li_lh[i] = kLiHash[i];
  for (uint32_t i = threadIdx.x; i < sizeof(kLiPool); i += blockDim.x) lid::li_lp[i] = kLiPool[i];
  __syncthreads();
  const lid::LiTables T{nullptr, nullptr, nullptr};  // (the copy reads lid::li_* itself)
  const uint32_t n = min(*B.det_count, B.det_cap);
  uint64_t dsteps = 0;  // value bytes through libinjection (secondary roofline)
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const DetEnt x = ((const DetEnt*)B.det)[e];
    GI_BOUND(x.req < B.n_req && x.off + x.len <= B.det_bytes_cap, x.req, x.off);
    const uint8_t* v = B.det_bytes + x.off;
    if (GI_DETECT_LVAL && x.len <= 64) {  // the arena offset is 16-byte aligned: four 16-byte loads
#if GI_DETECT_LVAL
      uint32_t* dst = lval + threadIdx.x * 17;
#else
      uint32_t* dst = nullptr;
#endif
      const uint4* src = (const uint4*)v;
      for (uint32_t k = 0; k < (x.len + 15) / 16; k++) {
        const uint4 w = src[k];
        dst[4 * k] = w.x;
        dst[4 * k + 1] = w.y;
        dst[4 * k + 2] = w.z;
        dst[4 * k + 3] = w.w;
      }
      v = (const uint8_t*)dst;
    }
    // which detectors the entry's admitting value tests need, then their
    // results (memoised across the batch), then the hit bits
    bool need_s = false, need_x = false;
    for (uint32_t d = 0; d < P.n_det_streams; d++) {
      if (!((x.mask >> d) & 1u)) continue;
      const DStream S = P.streams[P.det_streams[d]];
      const uint64_t fm = x.gm & S.gmask;
      for (uint32_t q = 0; q < S.val_count; q++) {
        const DScanVal sv = P.svals[S.val_begin + q];
        // (the body stage's entries are body fields: the prefix tests ran in the first stage)
        if (!(fm & sv.fmask) || (B.stage == 2 && sv.prefix)) continue;
        need_s = need_s || sv.kind == OP_DETECT_SQLI;
        need_x = need_x || sv.kind == OP_DETECT_XSS;
      }
    }
    const uint32_t res2 = det_results(B, v, x.len, x.off, need_s, need_x, &st[threadIdx.x], T, &dsteps);
    for (uint32_t d = 0; d < P.n_det_streams; d++) {
      if (!((x.mask >> d) & 1u)) continue;
      const DStream S = P.streams[P.det_streams[d]];
      const uint64_t fm = x.gm & S.gmask;
      for (uint32_t q = 0; q < S.val_count; q++) {
        const DScanVal sv = P.svals[S.val_begin + q];
        if (!(fm & sv.fmask) || (B.stage == 2 && sv.prefix)) continue;
        if (sv.kind != OP_DETECT_SQLI && sv.kind != OP_DETECT_XSS) continue;
        const bool res = (res2 >> (sv.kind == OP_DETECT_SQLI ? 0 : 1)) & 1u;
        if (res != (sv.negate != 0)) hit_value(B, sv.slot, x.req, x.vix);
      }
    }
  }
  dsteps = wave_sum(dsteps);
  if ((threadIdx.x & 63) == 0 && dsteps) atomicAdd(&B.acct2[5], (unsigned long long)dsteps);
}

// Slow values (non-ASCII / "maybe"), one thread per list entry: every job of
// the value's stream on the global tables.
__global__ void __launch_bounds__(256) k_scan_slow(DProgram P, DBatch B) {
  const uint32_t n = min(*B.slow_count, B.slow_cap);
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const SlowEnt x = ((const SlowEnt*)B.slow)[e];
    GI_BOUND(x.req < B.n_req && x.stream < P.n_streams && x.off + x.len <= B.slow_bytes_cap, x.req, x.stream);
    const DStream S = P.streams[x.stream];
    for (uint32_t j = S.job_begin; j < S.job_begin + S.job_count; j++)
      if (stage_runs(B, (x.flags & 2) != 0, P.jobs[j].prefix))
        scan_value_global(P, B, x.req, x.vix, P.jobs[j], x.fm, (x.flags & 1) != 0, B.slow_bytes + x.off, x.len);
  }
}

// ------------------------------------------------ stage 3: k_eval (phase B)
// RuleGroup.Eval(1) -> ProcessRequestBody -> RuleGroup.Eval(2) per request,
// skipping every phase-A rule whose hit bit is clear.
#ifndef GI_EVAL_WPE
#define GI_EVAL_WPE 1  // minimum waves per SIMD k_eval is compiled for (register budget).  Round 5, C2 A/B on
                       // one box: the Tx in registers (build_kindex no longer takes &t.nb) at 1 wave/SIMD, no
                       // spills: 25.5 ms; at 2 waves (418 VGPR spills) 30.0 ms; the Tx in scratch at 2: 27.6 ms
#endif
// Phase B of request r: RuleGroup.Eval(1) -> ProcessRequestBody ->
// RuleGroup.Eval(2); my[7] = its tally contributions.  W (k_eval_wave): the
// request's whole wave runs it uniformly, whits = the request's hit words in
// LDS (nullptr: read from HBM).
template <bool W>
GI_HD __forceinline__ void eval_request(const DProgram& Pk, const DBatch& B, uint32_t r, const uint32_t* whits,
                                             uint32_t wstride, unsigned long long* my) {
  // The interpreter reads the program through B.prog, a copy of the kernel's
  // DProgram in device memory: the non-inlined helpers take it by reference,
  // and a reference to the by-value kernel argument would make every lane copy
  // the whole struct into its scratch at entry (and read it back from there).
  (void)Pk;
  const DProgram& P = *B.prog;
  const uint64_t c_start = B.prof ? gi_clock() : 0;
  const gi_request rq = B.reqs[r];
  Region g = region_of(P, B, r);
  ReqHdr* H = g.hdr;
  Tx t;
  t.prof_visits = t.prof_evals = t.prof_rules = t.prof_ops = 0;
  t.prof_eval_cyc = t.prof_act_cyc = 0;
  const bool lead = !W || (gi_tid() & 63u) == 0;  // the lane that writes shared counters
  t.profon = B.prof != nullptr && lead;
  t.prof_rule_cyc = B.prof ? B.prof + 128 : nullptr;
  tx_bind(t, P, g);
  t.hits = whits ? whits : B.hits + r;
  t.hstride = whits ? wstride : B.rstride;
  t.vmap = B.vmap + B.layout[r].vmap_bit;
  {
    const ReqLayout Lr = B.layout[r];
    const uint32_t* tab = B.hset + Lr.hset_word;
    t.hset = (Lr.hset_mask && tab[0] == 0u) ? tab : nullptr;
    t.hmask = Lr.hset_mask;
  }
  t.nf_pa = H->nf;
  t.n_req = B.rstride;  // TX slot stride
  t.req = r;
  t.slots = B.txslots + r;
  t.has_post = false;
  t.body_spec = false;
  t.pa_void = H->pa_void != 0;
  t.nf = H->nf;
  t.nb = H->nb;
  t.flags = H->flags;
  t.body_proc = H->body_proc;
  t.ntx = 0;
  t.nremoved = 0;
  t.nrtgt = 0;
  t.rm_groups = 0;
  t.cur_groups = 0;
  t.allow = 0;
  t.prefix = false;
  t.prefix_spec = false;
  t.bail = false;
  t.kx = nullptr;
  t.engine = P.rule_engine;
  t.body_access = P.body_access;
  t.force_body = 0;
  t.phase = 0;
  t.skip_after = -1;
  t.skip = 0;
  t.interrupted = false;
  t.int_rule = 0;
  t.int_status = 0;
  t.int_action = 0;
  t.int_phase = 0;
  t.nmatched = 0;
  t.mout = B.matched + (uint64_t)r * B.mcap;
  t.cur_id = 0;
  if (t.capws) {
    CapHdr* CH = (CapHdr*)t.capws;
    CH->nrec = CH->nbytes = 0;
    CH->rec = B.caprec ? B.caprec + 4ull * B.crcap * r : nullptr;
    CH->bytes = B.capbytes ? B.capbytes + (uint64_t)B.cbcap * r : nullptr;
    CH->rec_cap = B.crcap;
    CH->bytes_cap = B.cbcap;
    CH->trunc = 0;
  }
  t.crec = t.capws && B.caprec;
  t.rcoll = false;
  t.rbody = false;
  t.mcap = B.mcap;
  // TX: copy on write over the folded snapshot; slots >= 128 and the capture
  // groups (run_capture writes those directly) start owned and unset
  t.wm0 = t.wm1 = 0;
  t.snap = false;
  for (uint32_t s = 128; s < P.n_slots; s++) TXS(t, s).state = 0;
  if (t.capws)
    for (uint32_t g = 0; g < 9; g++) {
      const int32_t cs = P.cap_slots[g];
      if (cs >= 0) {
        TXS(t, cs).state = 0;
        if (cs < 64) t.wm0 |= 1ull << cs;
        else if (cs < 128) t.wm1 |= 1ull << (cs - 64);
      }
    }
  if (t.dyn) {
    const ReqLayout Lr = B.layout[r];
    *(DynHdr*)t.dyn = DynHdr{0u, Lr.dyn_cap, 0u, Lr.dyn_capb};
  }
  if (t.mv) {
    const ReqLayout Lm = B.layout[r];
    t.mv->n = t.mv->nb = 0;
    t.mv->keep = 0;
    t.mv->cur = 0;
    t.mv->cap_e = Lm.mv_cap_e;
    t.mv->cap_a = Lm.mv_cap_a;
    t.mv->cap_v = g.cap_t;
    t.mv->cap_n = g.cap_mt;
    t.mv->cur_vn = t.mv->cur_nn = 0;
  }
  const uint8_t* D = B.data;
  uint64_t scanned = (uint64_t)rq.method.len + rq.uri.len + rq.proto.len + rq.body.len;
  for (uint32_t h = 0; h < rq.hdr_count; h++) {
    const gi_header hd = B.headers[rq.hdr_begin + h];
    scanned += hd.name.len + hd.value.len;
  }
  t.kx = kindex_into(t.fields, t.nf, t.bytes, t.nb, t.cap_b);
  const uint64_t c_init = B.prof ? gi_clock() : 0;
  // the gate's first stage: phase A has not scanned the body fields yet, so a
  // request with a body runs phase 1 and the phase-2 rules before the first
  // one whose evaluation needs that scan (RF2_BODY_PA), with the body fields
  // evaluated by the interpreter (their hit bits void: has_post); reaching
  // that rule undecided, it continues in the body stage (launch_pipeline)
  const Str rbp0 = t.single[S_REQBODY_PROCESSOR];
  // phase 1, ProcessRequestBody, phase 2 (one eval_phase call site)
  for (uint8_t ph = 1; ph <= 2 && !(t.flags & GI_REQ_ERROR_MASK); ph++) {
    if (ph == 2) {
      if (t.interrupted || t.engine == ENGINE_OFF) break;
      uint32_t bn = rq.body.len;
      bool run2 = true;
      if (t.body_access && bn > 0) {
        // [upstream transaction.go WriteRequestBody]: over SecRequestBodyLimit
        // -> INBOUND_DATA_ERROR; Reject: interruption 413 (no rule id) and no
        // ProcessRequestBody; ProcessPartial: the first limit bytes.
        // ProcessRequestBody: a buffer of exactly the limit sets it too and,
        // with Reject, returns before phase 2.  (DetectionOnly + Reject:
        // nothing buffered.)
        if (bn > P.body_limit) {
          t.single[S_INBOUND_DATA_ERROR] = {CS_ONE, 1};
          if (!P.body_partial) {
            if (t.engine == ENGINE_ON) {
              t.interrupted = true;
              t.int_rule = 0;
              t.int_status = 413;
              t.int_action = GI_ACTION_DENY;
              t.int_phase = 2;
              break;
            }
            bn = 0;
          } else {
            bn = (uint32_t)P.body_limit;
          }
        }
        if (bn > 0 && bn >= P.body_limit) {
          t.single[S_INBOUND_DATA_ERROR] = {CS_ONE, 1};
          if (!P.body_partial) run2 = false;
        }
      }
      if (t.body_access && bn > 0 && run2) {
        {
          uint8_t* lb = tx_alloc(t, 24);
          if (lb) t.single[S_REQUEST_BODY_LENGTH] = {lb, go_itoa((int64_t)bn, lb)};
          if (t.force_body && t.body_proc == BP_NONE) {
            t.body_proc = BP_URLENCODED;
            t.single[S_REQBODY_PROCESSOR] = {CS_URLENCODED, 10};
          }
          if (t.body_proc == BP_URLENCODED || t.body_proc == BP_JSON) {
            t.single[S_REQUEST_BODY] = {D + rq.body.off, bn};
            if (t.body_proc == H->spec_proc && B.stage == 1) {
              t.nf += H->n_post;  // k_bparse's fields: scanned through the prefix streams only
              t.nf_pa = t.nf;      // (value map valid for RF2_PREFIX links; the others' bits are void)
              t.has_post = H->n_post > 0;
              t.prefix_spec = true;
              t.body_spec = true;  // k_body (first stage) tested REQUEST_BODY
            } else if (t.body_proc == H->spec_proc) {
              t.nf += H->n_post;  // k_bparse's fields, already in phase A
              t.nf_pa = t.nf;
              t.body_spec = true;
            } else {
              const uint32_t nf0 = t.nf;
              if (t.body_proc == BP_URLENCODED) parse_query(t, D + rq.body.off, bn, FK_ARG_POST);
              else {
                JsonCtx jc{t.fields, t.nf, t.cap_f, t.bytes, t.nb, t.cap_b, t.t1, t.cap_t, t.flags};
                parse_json_body_ool(&jc, D + rq.body.off, bn);
                t.nf = jc.nf;
                t.nb = jc.nb;
                t.flags = jc.flags;
                if (t.flags & GI_REQ_BODY_ERROR) {
                  // readJSON's error -> generateRequestBodyError: REQBODY_ERROR "1",
                  // REQBODY_ERROR_MSG "<processor>: <error>", no ARGS_POST, no REQUEST_BODY;
                  // phase 2 still runs (CRS base rule 200002 denies with 400)
                  t.nf = nf0;
                  t.single[S_REQBODY_ERROR] = {CS_ONE, 1};
                  t.single[S_REQBODY_ERROR_MSG] = {CS_JSON_ERR, 18};
                  t.single[S_REQUEST_BODY] = {CS_ZERO, 0};
                }
              }
              t.has_post = t.nf > nf0;
            }
          } else if (t.body_proc == BP_MULTIPART) {
            // [upstream multipart.go]: collections, no REQUEST_BODY; an error
            // -> MULTIPART_STRICT_ERROR + generateRequestBodyError (rules
            // 200002 / 200003 deny with 400)
            t.rcoll = true;  // part headers (MULTIPART_PART_HEADERS) and FILES_TMPNAMES
            uint8_t err;
            if (H->spec_proc == BP_MULTIPART && B.stage == 1) {
              t.nf += H->n_post;  // k_mpparse's fields: scanned through the prefix streams only
              t.nf_pa = t.nf;
              t.has_post = H->n_post > 0;
              t.prefix_spec = true;
              err = H->spec_err;
            } else if (H->spec_proc == BP_MULTIPART) {
              t.nf += H->n_post;  // k_mpparse's fields (ARGS_POST already in phase A)
              t.nf_pa = t.nf;
              t.body_spec = true;
              err = H->spec_err;
            } else {
              const uint32_t nf0 = t.nf;
              JsonCtx jc{t.fields, t.nf, t.cap_f, t.bytes, t.nb, t.cap_b, t.t1, t.cap_t, t.flags};
              const Str ct = first_content_type(B, rq);
              uint64_t comb;
              bool comb_set;
              err = parse_multipart(jc, D + rq.body.off, bn, ct.p, ct.n, &comb, &comb_set);
              t.nf = jc.nf;
              t.nb = jc.nb;
              t.flags = jc.flags;
              if (comb_set && !(t.flags & GI_REQ_ERROR_MASK)) {
                uint8_t* cb = tx_alloc(t, 24);
                if (cb) t.single[S_FILES_COMBINED_SIZE] = {cb, go_itoa((int64_t)comb, cb)};
              }
              t.has_post = t.nf > nf0;
            }
            if (err) {
              t.single[S_MULTIPART_STRICT_ERROR] = {CS_ONE, 1};
              t.single[S_REQBODY_ERROR] = {CS_ONE, 1};
              t.single[S_REQBODY_ERROR_MSG] = mp_err_msg(err);
            }
          } else if (t.body_proc == BP_XML) {
            // [upstream xml.go]: XML "//@*" / "/*", no REQUEST_BODY; an error ->
            // generateRequestBodyError (REQBODY_ERROR_MSG "XML: <error>")
            t.rcoll = true;
            JsonCtx jc{t.fields, t.nf, t.cap_f, t.bytes, t.nb, t.cap_b, t.t1, t.cap_t, t.flags};
            Str msg{CS_ZERO, 0};
            const int xr = parse_xml(jc, D + rq.body.off, bn, (uint32_t*)t.t0, t.cap_t / 4, &msg);
            t.nf = jc.nf;
            t.nb = jc.nb;
            t.flags = jc.flags;
            if (xr == 1) {
              t.single[S_REQBODY_ERROR] = {CS_ONE, 1};
              t.single[S_REQBODY_ERROR_MSG] = msg;
            }
          } else if (t.body_proc != BP_NONE) {
            t.flags |= GI_REQ_UNSUPPORTED_BODY;
          }
          if (t.nf != H->nf) t.kx = kindex_into(t.fields, t.nf, t.bytes, t.nb, t.cap_b);
        }
      }
      if ((t.flags & GI_REQ_ERROR_MASK) || !run2) break;
      t.rbody = t.single[S_REQUEST_BODY].n > 0;
      // (body fields or a REQUEST_BODY phase A has not seen: XML values are never phase-A items)
      t.prefix = B.stage == 1 && (t.has_post || t.single[S_REQUEST_BODY].n > 0);
    }
    const uint64_t c0 = B.prof ? gi_clock() : 0;
    eval_phase<W>(t, ph);
    if (B.prof && lead) gi_prof_add(&B.prof[ph], (unsigned long long)(gi_clock() - c0));
  }
  if (t.bail) {
    // undecided before a rule that needs the body's phase-A scan: the body
    // stage evaluates the request again from the start.  The request state
    // the phase-2 prologue wrote goes back to k_collect's / the parsers' values.
    if (lead) {
      t.single[S_REQBODY_PROCESSOR] = rbp0;
      t.single[S_INBOUND_DATA_ERROR] = {CS_ZERO, 0};
      t.single[S_REQUEST_BODY_LENGTH] = {CS_ZERO, 0};
      t.single[S_REQUEST_BODY] = {CS_ZERO, 0};
      t.single[S_REQBODY_ERROR] = {CS_ZERO, 1};
      t.single[S_REQBODY_ERROR_MSG] = {CS_ZERO, 0};
      t.single[S_MULTIPART_STRICT_ERROR] = {CS_ZERO, 1};
      if (H->spec_proc != BP_MULTIPART) t.single[S_FILES_COMBINED_SIZE] = {CS_ZERO, 0};
      B.pend[r] = 1;
      B.plist[gi_fetch_add(B.pcount, 1u)] = r;
      gi_fetch_add(B.pcount + 1, 1u);  // pending requests of the whole run (gi_stats.gate_pending)
    }
    for (int c = 0; c < 7; c++) my[c] = 0;
    return;
  }
  if (B.prof && lead) {
    gi_prof_add(&B.prof[0], (unsigned long long)(c_init - c_start));
    gi_prof_add(&B.prof[3], (unsigned long long)(gi_clock() - c_start));
    gi_prof_add(&B.prof[4], (unsigned long long)t.prof_visits);
    gi_prof_add(&B.prof[5], (unsigned long long)t.prof_evals);
    gi_prof_add(&B.prof[6], (unsigned long long)t.prof_rules);
    gi_prof_add(&B.prof[7], (unsigned long long)t.prof_eval_cyc);
    gi_prof_add(&B.prof[8], (unsigned long long)t.prof_act_cyc);
  }
  gi_verdict v;
  v.rule_id = t.interrupted ? t.int_rule : 0;
  v.status = t.interrupted ? t.int_status : 0;
  v.action = t.interrupted ? t.int_action : 0;
  v.phase = t.interrupted ? t.int_phase : 0;
  v.capture_cnt = 0;
  v._pad = 0;
  if (t.capws) {
    const CapHdr* CH = (const CapHdr*)t.capws;
    v.capture_cnt = CH->nrec;
    if (CH->trunc) t.flags |= GI_REQ_CAPTURE_TRUNC;
  }
  v.flags = t.flags;
  v.match_cnt = t.nmatched;
  for (uint32_t e = 0; e < GI_MAX_EXPORTS; e++) {
    int64_t x = 0;
    if (e < P.n_exports && P.exports[e] >= 0) {
      bool okk;
      x = slot_int(slot_rd(t, (uint32_t)P.exports[e]), &okk);
      if (!okk) x = 0;
    }
    v.tx_export[e] = x;
  }
  if (lead) {
    B.verdicts[r] = v;
    if (B.stage == 1) B.pend[r] = 0;
  }
  my[0] = 1;
  my[1] = t.interrupted ? 1 : 0;
  my[2] = t.nmatched ? 1 : 0;
  my[3] = (t.flags & GI_REQ_ERROR_MASK) ? 1 : 0;
  my[4] = scanned;
  my[5] = t.nmatched;
  my[6] = t.pa_void ? 1 : 0;
}

// Requests k_eval hands to k_eval_wave: many fields (a POST body's
// ARGS_POST, multipart collections) or a large program (rule walks of
// thousands of rules), where the lanes of one wave split the field loops and
// the rule walk instead of one lane doing both alone.
GI_HD __forceinline__ bool eval_heavy(const DProgram& P, const DBatch& B, uint32_t r) {
  if (!B.wlist) return false;
  // the gate's body stage: its few pending requests are the heavy ones (long
  // bodies, every body rule still to run), one lane each would leave most of
  // the GPU idle -- a wave each (DBatch.wave_stage2, GI_EVAL_WAVE_STAGE2)
  if (B.stage == 2 && B.wave_stage2) return true;
  if (B.wave_rules && P.top_end[1] - P.top_begin[0] >= B.wave_rules) return true;
  const ReqHdr* H = (const ReqHdr*)(B.scratch + B.layout[r].base);
  return B.wave_fields && H->nf + H->n_post >= B.wave_fields;
}

// k_eval's request order.  A wave of k_eval runs its 64 requests' rule walks
// in lockstep, so one request with many set hit bits (an attack: detectors,
// chains and actions to re-run) holds the other 63 lanes; with 5 % attacks
// nearly every wave has one.  Grouping requests by their number of set
// phase-A hit bits (a counting sort into GI_EORD_BINS bins; void requests,
// which evaluate every link, in the last) gives waves of like requests.  The
// order changes no result: each request is evaluated on its own.
// (k_eord_count keeps each request's bin in eord_key[r] for k_eord_scatter.)
GI_HD __forceinline__ uint32_t eord_key(const DBatch& B, uint32_t r) {
  const uint32_t nw = (B.n_hit_slots + 31) / 32;
  uint32_t c = 0;
  for (uint32_t w = 0; w < nw; w++) c += __popc(B.hits[(uint64_t)w * B.rstride + r]);
  // most set bits first: the heaviest waves start first and the light ones
  // fill the tail (longest-processing-time-first across the CUs)
  return (uint32_t)GI_EORD_BINS - 1 - min(c, (uint32_t)GI_EORD_BINS - 1);
}
// Both launches run GI_EORD_GRID workgroups, each over one contiguous chunk of
// requests, with the bins counted in LDS: one global atomic per (workgroup,
// bin) instead of one per (wave, bin) on 32 hot counters.
__device__ __forceinline__ void eord_chunk(const DBatch& B, uint32_t* r0, uint32_t* r1) {
  const uint32_t per = (B.n_req + gridDim.x - 1) / gridDim.x;
  *r0 = min(B.n_req, blockIdx.x * per);
  *r1 = min(B.n_req, *r0 + per);
}
__global__ void __launch_bounds__(256) k_eord_count(DBatch B) {
  __shared__ uint32_t h[GI_EORD_BINS];
  if (threadIdx.x < GI_EORD_BINS) h[threadIdx.x] = 0;
  __syncthreads();
  uint32_t r0, r1;
  eord_chunk(B, &r0, &r1);
  for (uint32_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const uint32_t key = eord_key(B, r);
    B.eord_key[r] = (uint8_t)key;
    atomicAdd(&h[key], 1u);
  }
  __syncthreads();
  if (threadIdx.x < GI_EORD_BINS && h[threadIdx.x]) atomicAdd(&B.eord_bins[threadIdx.x], h[threadIdx.x]);
}
__global__ void __launch_bounds__(256) k_eord_scatter(DBatch B) {
  __shared__ uint32_t h[GI_EORD_BINS], base[GI_EORD_BINS];
  if (threadIdx.x < GI_EORD_BINS) h[threadIdx.x] = 0;
  __syncthreads();
  uint32_t r0, r1;
  eord_chunk(B, &r0, &r1);
  for (uint32_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) atomicAdd(&h[B.eord_key[r]], 1u);
  __syncthreads();
  if (threadIdx.x < GI_EORD_BINS) {  // this workgroup's run of each bin
    uint32_t a = 0;
    for (uint32_t k = 0; k < threadIdx.x; k++) a += B.eord_bins[k];
    base[threadIdx.x] = a + (h[threadIdx.x] ? atomicAdd(&B.eord_bins[GI_EORD_BINS + threadIdx.x], h[threadIdx.x]) : 0u);
    h[threadIdx.x] = 0;
  }
  __syncthreads();
  for (uint32_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const uint32_t key = B.eord_key[r];
    B.eorder[base[key] + atomicAdd(&h[key], 1u)] = r;
  }
}

__global__ void __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(GI_EVAL_WPE, 8))) k_eval(DProgram P, DBatch B) {
  __shared__ unsigned long long red[7];
  // the block's hit words in LDS ([word][thread]): the rule walk tests one per
  // rule, and an LDS read waits far less than a global one
  __shared__ uint32_t lhits[GI_EVAL_LDS_WORDS * 128];
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x < 7) red[threadIdx.x] = 0;
  const uint32_t nw = (B.n_hit_slots + 31) / 32;
  const bool in_lds = nw <= GI_EVAL_LDS_WORDS && blockDim.x <= 128;
  // the gate's body stage: the pending requests of the phase-1 stage, in its
  // list; otherwise k_eord's order when there is one
  const uint32_t rr = B.stage == 2 ? (r < *B.pcount ? B.plist[r] : 0xFFFFFFFFu)
                      : (B.eorder && r < B.n_req) ? B.eorder[r] : r;
  if (in_lds && rr < B.n_req)
    for (uint32_t w = 0; w < nw; w++) lhits[w * blockDim.x + threadIdx.x] = B.hits[(uint64_t)w * B.rstride + rr];
  __syncthreads();
  unsigned long long my[7] = {0, 0, 0, 0, 0, 0, 0};
  if (rr < B.n_req) {
    if (eval_heavy(P, B, rr)) B.wlist[atomicAdd(B.wcount, 1u)] = rr;
    else eval_request<false>(P, B, rr, in_lds ? lhits + threadIdx.x : nullptr, blockDim.x, my);
  }
  for (int c = 0; c < 7; c++) {
    unsigned long long x = my[c];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[c], x);
  }
  __syncthreads();
  if (threadIdx.x < 7) atomicAdd(&B.tally[threadIdx.x], red[threadIdx.x]);
}

// One wave per heavy request (k_eval's list), persistent over the list.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GI_EVAL_WPE, 8))) k_eval_wave(DProgram P, DBatch B) {
  extern __shared__ uint32_t whits[];
  const uint32_t lane = threadIdx.x;
  const uint32_t nw = (B.n_hit_slots + 31) / 32;
  const bool in_lds = nw <= GI_EVAL_WAVE_LDS_WORDS;
  unsigned long long acc[7] = {0, 0, 0, 0, 0, 0, 0};
  const uint32_t n = min(*B.wcount, B.n_req);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t r = B.wlist[i];
    GI_BOUND(r < B.n_req, r, i);
    if (in_lds) {
      __syncthreads();
      for (uint32_t w = lane; w < nw; w += 64) whits[w] = B.hits[(uint64_t)w * B.rstride + r];
      __syncthreads();
    }
    unsigned long long my[7] = {0, 0, 0, 0, 0, 0, 0};
    eval_request<true>(P, B, r, in_lds ? whits : nullptr, 1u, my);
    for (int c = 0; c < 7; c++) acc[c] += my[c];
  }
  if (lane == 0)
    for (int c = 0; c < 7; c++)
      if (acc[c]) atomicAdd(&B.tally[c], acc[c]);
}

// Detail tally: histogram of the exported inbound score (DProgram.hist_mask) and
// the match count of every rule id, from the verdicts and matched-id rows k_eval
// wrote.  A wave takes 64 requests: the score bins lane-per-request (equal bins
// aggregated across the wave: one atomic per distinct bin), then the 64
// matched-id rows as one flattened list, 64 consecutive entries per step.
GI_HD __forceinline__ void wave_hist_add(uint32_t* hist, int32_t b) {
  uint64_t active = __ballot(b >= 0);
  while (active) {
    const int leader = __ffsll((unsigned long long)active) - 1;
    const int32_t lb = __shfl(b, leader, 64);
    const uint64_t same = __ballot(b == lb) & active;
    if (lane_id() == (uint32_t)leader) atomicAdd(&hist[lb], (uint32_t)__popcll(same));
    active &= ~same;
  }
}

__global__ void __launch_bounds__(256) k_tally(DBatch B, const uint32_t* __restrict__ ids, uint32_t n_ids,
                                               uint32_t hist_mask) {
  extern __shared__ uint32_t sh[];  // [n_ids] sorted ids | [GI_SCORE_BINS + n_ids] counts (LDS mode)
  const bool lds = n_ids <= GI_RHIST_LDS;
  const uint32_t* tid = lds ? sh : ids;
  uint32_t* hist = lds ? sh + n_ids : B.tally_ext;
  if (lds) {
    for (uint32_t i = threadIdx.x; i < n_ids; i += blockDim.x) sh[i] = ids[i];
    for (uint32_t i = threadIdx.x; i < GI_SCORE_BINS + n_ids; i += blockDim.x) hist[i] = 0;
  }
  __syncthreads();
  // whole waves stay in the loop together (the aggregation uses ballots)
  const uint32_t n_waves_total = (B.n_req + 63) / 64;
  const uint32_t wv = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  const uint32_t stride_w = gridDim.x * blockDim.x / 64;
  for (uint32_t w = wv; w < n_waves_total; w += stride_w) {
    const uint32_t r = w * 64 + lane_id();
    uint32_t cnt = 0;
    int32_t sb = -1;
    if (r < B.n_req) {
      const gi_verdict v = B.verdicts[r];
      cnt = min(v.match_cnt, B.mcap);
      int64_t sc = 0;
      for (uint32_t e = 0; e < GI_MAX_EXPORTS; e++)  // terms clamped to +-2^50: the sum cannot overflow
        if ((hist_mask >> e) & 1u) sc += min(max(v.tx_export[e], -(1ll << 50)), 1ll << 50);
      sb = (int32_t)min(max(sc, (int64_t)0), (int64_t)(GI_SCORE_BINS - 1));
    }
    wave_hist_add(hist, sb);
    // The wave's 64 matched-id rows as one flattened list (inclusive prefix of
    // the counts across the lanes): lane i takes entry base + i, so a wave's
    // reads walk each row contiguously instead of 64 rows at one column.
    uint32_t incl = cnt;
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane_id() >= o) incl += y;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    const uint32_t excl = incl - cnt;
    for (uint32_t base = 0; base < total; base += 64) {
      const uint32_t j = base + lane_id();
      uint32_t lo = 0, hi = 63;  // owner: the first lane whose inclusive prefix exceeds j
      for (int it = 0; it < 6; it++) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t v = __shfl(incl, (int)mid, 64);
        if (lo < hi) {
          if (v > j) hi = mid;
          else lo = mid + 1;
        }
      }
      const uint32_t q_excl = __shfl(excl, (int)lo, 64);
      int32_t b = -1;
      if (j < total) {
        const uint32_t id = B.matched[(uint64_t)(w * 64 + lo) * B.mcap + (j - q_excl)];
        uint32_t a = 0, e = n_ids;
        while (a < e) {
          const uint32_t mid = (a + e) >> 1;
          if (tid[mid] < id) a = mid + 1;
          else e = mid;
        }
        if (a < n_ids && tid[a] == id) b = (int32_t)(GI_SCORE_BINS + a);
      }
      if (lds) {  // the lanes hold a few requests' lists: mostly distinct bins
        if (b >= 0) atomicAdd(&hist[b], 1u);
      } else {
        wave_hist_add(hist, b);
      }
    }
  }
  if (lds) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < GI_SCORE_BINS + n_ids; i += blockDim.x)
      if (hist[i]) atomicAdd(&B.tally_ext[i], hist[i]);
  }
}

void scan_allow_lds(uint32_t lds_bytes) {
  if (lds_bytes > 65536) {
    (void)hipFuncSetAttribute((const void*)k_scan<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_bytes);
    (void)hipFuncSetAttribute((const void*)k_scan<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_bytes);
  }
}

uint32_t scan_resident_blocks(uint32_t lds_bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, dev);
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_scan<true, false>, 1024, lds_bytes);
  if (per_cu < 1) per_cu = 1;
  return (uint32_t)prop.multiProcessorCount * (uint32_t)per_cu;
}

#define GI_LAUNCH(nm, ...)                                                                \
  do {                                                                                    \
    if (stop_after && nk + 1 > stop_after) return;                                        \
    nk++;                                                                                 \
    hipLaunchKernelGGL(__VA_ARGS__);                                                      \
    if (log && log->n < GI_MAX_LAUNCHES) {                                                \
      log->name[log->n] = nm;                                                             \
      (void)hipEventRecord(log->ev[++log->n], stream);                                    \
    }                                                                                     \
    if (stop_after) {                                                                     \
      hipError_t e_ = hipStreamSynchronize(stream);                                       \
      fprintf(stderr, "GI_STOP_AFTER: kernel %d %s -> %s\n", nk, nm, hipGetErrorString(e_));   \
      if (e_ != hipSuccess) return;                                                       \
    }                                                                                     \
  } while (0)

// CPU baseline ("the build's own C++ CPU restatement", not
// Coraza): request 0 of B through the same interpreter, compiled for the
// host.  ProcessURI / headers / cookies (collect_request), then phase B with
// phase A void -- every rule link evaluated by the interpreter, the body
// parsed in phase B -- and the verdict, matched ids and exports in B.
void cpu_inspect_one(const DProgram& P, const DBatch& B) {
  collect_request(P, B, 0);
  ReqHdr* H = (ReqHdr*)(B.scratch + B.layout[0].base);
  H->spec_proc = BP_NONE;
  H->pa_void = 1;
  unsigned long long my[8];
  eval_request<false>(P, B, 0, nullptr, 0, my);
}

// The copies' phase-A results from their canonical occurrences (hdr_dedup),
// one thread per request, after every phase-A producer of the stage.
__global__ void __launch_bounds__(256) k_dspread(DProgram P, DBatch B) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B.n_req) return;
  const ReqLayout L = B.layout[r];
  const ReqHdr* H = (const ReqHdr*)(B.scratch + L.base);
  if (H->flags & GI_REQ_ERROR_MASK) return;
  const Field* Fd = (const Field*)(B.scratch + L.base + GI_REQHDR_BYTES);
  const gi_request rq = B.reqs[r];
  bool voided = false;
  uint32_t hx = 0;
  for (uint32_t i = H->n_get; i < H->n_get + H->n_hdr && !voided; i++) {
    while (hx < rq.hdr_count && B.headers[rq.hdr_begin + hx].name.len == 0) hx++;
    const uint32_t g = rq.hdr_begin + hx++;
    const Field fl = Fd[i];
    for (uint32_t side = 0; side < 2 && !voided; side++) {
      if (!((fl._pad >> side) & 1u)) continue;
      const uint32_t e1 = B.hdref[2ull * g + side];
      bool ok = e1 != 0 && e1 - 1u <= B.hdmask;
      uint32_t r0 = 0, f0 = 0;
      if (ok) {  // (published before hdr_dedup recorded it: k_collect, a launch earlier)
        const unsigned long long inf = B.hdinfo[e1 - 1u];
        r0 = hd_info_req(inf);
        f0 = hd_info_fs(inf) >> 1;
        ok = inf != 0 && r0 < B.n_req;
      }
      ReqLayout L0{};
      const uint32_t* tab0 = nullptr;
      if (ok) {
        L0 = B.layout[r0];
        const ReqHdr* H0 = (const ReqHdr*)(B.scratch + L0.base);
        tab0 = B.hset + L0.hset_word;
        ok = !H0->pa_void && !(H0->flags & GI_REQ_ERROR_MASK) && L0.hset_mask && tab0[0] == 0u;
      }
      if (!ok) {  // the canonical's results are not exactly known: evaluate this request in full
        void_request(B, r, GI_VOID_DEDUP);
        voided = true;
        continue;
      }
      const uint32_t vix0 = 2u * f0 + side, vix = 2u * i + side;
      GI_BOUND(vix0 < L0.vmap_bits && vix < L.vmap_bits, vix0, vix);
      const uint32_t vb = B.vmap[L0.vmap_bit + vix0];
      if (!vb) continue;
      atomicOr(&B.vmap[L.vmap_bit + vix], vb);
      for (uint32_t m = vb; m; m &= m - 1) {
        for (uint32_t s = (uint32_t)(__ffs(m) - 1); s < B.n_hit_slots; s += 32) {
          const uint32_t res = hset_lookup(tab0, L0.hset_mask, s, vix0);
          if (!res) continue;
          set_hit(B, s, r);
          if (L.hset_mask) hset_insert(B, L, s, vix, res == 2 ? 1u : 0u);
        }
      }
    }
  }
}

// Phase A over the items of the current stage: item records, the streams'
// transformation chains, libinjection, long values and the automaton scans.
static void launch_phase_a(const DProgram& P, const DBatch& B, const ScanLaunch& S, hipStream_t stream,
                           hipEvent_t* ev, int stop_after, LaunchLog* log, int& nk) {
  const uint32_t cb = (B.n_req + 255) / 256;
  const bool s2 = B.stage == 2;  // the gate's body stage: its launches are timed under their own names
  GI_LAUNCH(s2 ? "k_ioffsets.2" : "k_ioffsets", k_ioffsets, dim3(GI_NCLS), dim3(256), 0, stream, B, cb);
  GI_LAUNCH(s2 ? "k_ibases.2" : "k_ibases", k_ibases, dim3(1), dim3(256), 0, stream, B);
  GI_LAUNCH(s2 ? "k_items.2" : "k_items", k_items, dim3(cb), dim3(256), 0, stream, P, B);
  // chain memo slots per lane: as many as keep 8 one-wave workgroups per CU within the LDS
  GI_LAUNCH(s2 ? "k_stream0.2" : "k_stream0", (k_stream<16, 20, 4>), dim3(GI_STREAM_GRID), dim3(64), 0, stream, P, B, 0u);
  GI_LAUNCH(s2 ? "k_stream1.2" : "k_stream1", (k_stream<32, 36, 3>), dim3(GI_STREAM_GRID), dim3(64), 0, stream, P, B, 1u);
  GI_LAUNCH(s2 ? "k_stream2.2" : "k_stream2", (k_stream<64, 68, 1>), dim3(GI_STREAM_GRID), dim3(64), 0, stream, P, B, 2u);
  GI_LAUNCH(s2 ? "k_stream3.2" : "k_stream3", (k_stream<128, 132, 0>), dim3(GI_STREAM_GRID), dim3(64), 0, stream, P, B, 3u);
  GI_LAUNCH(s2 ? "k_stream4.2" : "k_stream4", (k_stream<0, 0, 0>), dim3(GI_STREAM_GRID), dim3(64), 0, stream, P, B, 4u);
  if (P.n_det_streams) {
    if (B.dmemo_keys) {  // the det arena restarts: keys AND result words (a reader that sees a fresh claimer's
      // key before the claimer's info store must find w == 0, never the previous stage's or batch's VALID bits)
      (void)hipMemsetAsync(B.dmemo_keys, 0, 8ull * (B.dmemo_mask + 1), stream);
      (void)hipMemsetAsync(B.dmemo_info, 0, 16ull * (B.dmemo_mask + 1), stream);
    }
    // grid: 12 rounds of resident workgroups (3 per CU at 48 KB of LDS x 256
    // CUs): finer grid-stride shares balance the divergent detectors.  C2 A/B
    // (GI_DETECT_GRID): 768 11.9 ms, 2048 10.9, 3072 10.7, 6144 10.2, 9216 10.1
    static const uint32_t det_grid = getenv("GI_DETECT_GRID") ? (uint32_t)atoi(getenv("GI_DETECT_GRID")) : 9216u;
    GI_LAUNCH(s2 ? "k_detect.2" : "k_detect", k_detect, dim3(det_grid), dim3(256), 0, stream, P, B);
  }
  if (B.long_cap) GI_LAUNCH(s2 ? "k_long.2" : "k_long", k_long, dim3(B.long_grid), dim3(64), 0, stream, P, B);
  if (ev) (void)hipEventRecord(ev[1], stream);
  for (int big = 0; big < 2; big++)
    if (S.n_jobs[big]) {
      if (big)
        GI_LAUNCH(s2 ? "k_scan_big.2" : "k_scan_big", (k_scan<true, true>), dim3(S.blocks[big]), dim3(1024), S.lds[big], stream, P, B,
                  S.jobs[big], S.n_jobs[big], S.mode, 1u);
      else
        GI_LAUNCH(s2 ? "k_scan.2" : "k_scan", (k_scan<true, false>), dim3(S.blocks[big]), dim3(1024), S.lds[big], stream, P, B,
                  S.jobs[big], S.n_jobs[big], S.mode, 0u);
    }
  if (S.n_global)
    GI_LAUNCH(s2 ? "k_scan_hbm.2" : "k_scan_hbm", (k_scan<false, false>), dim3(S.blocks[2]), dim3(1024), 0, stream, P, B, S.global_jobs,
              S.n_global, S.mode, 2u);
  GI_LAUNCH(s2 ? "k_scan_slow.2" : "k_scan_slow", k_scan_slow, dim3(1024), dim3(256), 0, stream, P, B);
  // (the copies are header sides: phase-1 items, all scanned in the first / only stage)
  if (B.hdkeys && !s2) GI_LAUNCH("k_dspread", k_dspread, dim3((B.n_req + 255) / 256), dim3(256), 0, stream, P, B);
}

static void launch_eval(const DProgram& P, const DBatch& B, hipStream_t stream, int stop_after, LaunchLog* log,
                        int& nk) {
  DBatch Be = B;
  // the order pays on header-only traffic (C2: k_eval 15.2 -> 12.8 ms); with bodies in more than
  // 1 of 8 requests the waves of many-field requests it builds cost more (C3: 170 -> 259 ms)
  if (B.n_req < 4096 || B.stage == 2 || 8ull * B.n_body > B.n_req) Be.eorder = nullptr;
  if (Be.eorder) {
    const uint32_t cb = (B.n_req + 255) / 256;
    (void)hipMemsetAsync(B.eord_bins, 0, 8 * GI_EORD_BINS, stream);
    const uint32_t eg = std::min<uint32_t>(cb, GI_EORD_GRID);
    GI_LAUNCH(B.stage == 1 ? "k_eord_count.1" : "k_eord_count", k_eord_count, dim3(eg), dim3(256), 0, stream, B);
    GI_LAUNCH(B.stage == 1 ? "k_eord_scatter.1" : "k_eord_scatter", k_eord_scatter, dim3(eg), dim3(256), 0, stream, B);
  }
  {  // small batches (fewer than 4 workgroups of 128 per CU): one wave per workgroup to spread over all CUs
    // GI_EVAL_BS A/B (C2, 1M): 128 threads 26.2 ms, 64 threads 32.1 ms
    static const uint32_t ev_env = getenv("GI_EVAL_BS") ? (uint32_t)atoi(getenv("GI_EVAL_BS")) : 0u;
    const uint32_t ev_bs = (ev_env == 64 || ev_env == 128) ? ev_env : (B.n_req + 127) / 128 < 1024 ? 64u : 128u;
    GI_LAUNCH(B.stage == 2 ? "k_eval.2" : "k_eval", k_eval, dim3((B.n_req + ev_bs - 1) / ev_bs), dim3(ev_bs), 0, stream, P,
              Be);
  }
  if (B.wlist) {  // heavy requests, one wave each (persistent over k_eval's list)
    const uint32_t nw = (B.n_hit_slots + 31) / 32;
    const uint32_t lds = nw <= GI_EVAL_WAVE_LDS_WORDS ? 4 * std::max<uint32_t>(nw, 1u) : 0u;
    GI_LAUNCH(B.stage == 2 ? "k_eval_wave.2" : "k_eval_wave", k_eval_wave, dim3(std::min<uint32_t>(B.n_req, 8192)),
              dim3(64), lds, stream, P, B);
  }
}

void launch_pipeline(const DProgram& P, const DBatch& B0, const ScanLaunch& S, hipStream_t stream, hipEvent_t* ev,
                     int stop_after, LaunchLog* log, const uint32_t* tally_ids, uint32_t n_tally_ids) {
  if (!B0.n_req) return;
  int nk = 0;  // (the caller resets *log and records its ev[0] before the first chunk)
  const uint32_t cb = (B0.n_req + 255) / 256;
  // The gate: when the batch has bodies, the first stage parses them and runs
  // k_body's prefix links (REQUEST_BODY) but scans only the phase-1 items, and
  // evaluates every request up to the first phase-2 rule that needs its body
  // fields' phase-A scan (RF2_BODY_PA): requests with no body, and those phase
  // 1 or the phase-2 rules before it decide (CRS's ARGS-count / byte-range
  // checks, REQBODY_ERROR), are final there.  The second stage scans the other
  // (pending) requests' body fields and evaluates them in full.
  const bool gated = B0.gate && B0.n_body && P.body_access && B0.pend && B0.plist && B0.pcount;
  DBatch B = B0;
  B.stage = gated ? 1u : 0u;
  if (gated) (void)hipMemsetAsync(B.pcount, 0, 4, stream);
  GI_LAUNCH("k_collect", k_collect, dim3(cb), dim3(256), 0, stream, P, B);
  if (B.n_body && P.body_access) {
    GI_LAUNCH("k_bparse", k_bparse, dim3(std::min<uint32_t>(B.n_body, 1u << 20)), dim3(64), B.bparse_lds, stream, P, B);
    if (B.n_mp_body) GI_LAUNCH("k_mpparse", k_mpparse, dim3(std::min<uint32_t>(B.n_body, 1u << 20)), dim3(GI_MP_T), 0, stream, P, B);
  }
  if (ev) (void)hipEventRecord(ev[0], stream);
  if (P.n_streams) launch_phase_a(P, B, S, stream, ev, stop_after, log, nk);
  else if (ev) (void)hipEventRecord(ev[1], stream);
  if (stop_after && nk >= stop_after) return;
  // REQUEST_BODY links (a ruleset may have them without any phase-A stream):
  // one wave (workgroup) per body
  if (P.n_body_links && B.n_body)
    GI_LAUNCH("k_body", k_body, dim3(std::min<uint32_t>(B.n_body, 1u << 20)), dim3(64), 0, stream, P, B);
  if (ev) (void)hipEventRecord(ev[2], stream);
  launch_eval(P, B, stream, stop_after, log, nk);
  if (gated) {
    // the body stage: phase-A counters restart (the hit words, value
    // signatures and hit sets keep the first stage's bits)
    DBatch B2 = B0;
    B2.stage = 2;
    (void)hipMemsetAsync((void*)B2.pool_used, 0, 128, stream);  // ctr[0, 128): pool, slow, detect, long, wave list, buckets
    if (P.n_streams) {
      GI_LAUNCH("k_bcounts", k_bcounts, dim3(cb), dim3(256), 0, stream, P, B2);
      launch_phase_a(P, B2, S, stream, nullptr, stop_after, log, nk);
    }
    if (P.n_body_links) GI_LAUNCH("k_body.2", k_body, dim3(std::min<uint32_t>(B2.n_body, 1u << 20)), dim3(64), 0, stream, P, B2);
    launch_eval(P, B2, stream, stop_after, log, nk);
  }
  {
    const uint32_t lds = n_tally_ids <= GI_RHIST_LDS ? 4 * (2 * n_tally_ids + GI_SCORE_BINS) : 0;
    const uint32_t nb = std::min<uint32_t>((B.n_req + 255) / 256, 2048);
    GI_LAUNCH("k_tally", k_tally, dim3(nb), dim3(256), lds, stream, B, tally_ids, n_tally_ids, P.hist_mask);
  }
}

}  // namespace gi
