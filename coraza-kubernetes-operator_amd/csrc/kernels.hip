// HIP kernels of the inspection engine (gfx950).
//
// v1 pipeline = one launch, one thread per request ("transaction lane"):
//   collect  : ProcessURI + AddRequestHeader (query/cookie parsing, Go
//              net/url re-encoding of REQUEST_URI) into a per-request field
//              table in HBM scratch
//   phase 1  : RuleGroup.Eval(1) -- the rule interpreter below
//   body     : ProcessRequestBody (URLENCODED -> ARGS_POST)
//   phase 2  : RuleGroup.Eval(2)
//   verdict  : Interruption + matched rule ids + exported TX scores,
//              block-reduced tallies (one atomic per block per counter)
// Semantics follow coraza/v3 v3.3.3 [upstream, see DESIGN.md]; every
// function names the coraza source it restates.
#include <hip/hip_runtime.h>

#include "gi_kernels.h"

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

struct Slot {
  int64_t num;
  const uint8_t* p;
  uint32_t n;
  uint32_t state;  // 0 unset, 1 integer (canonical decimal), 2 string
};

__device__ __constant__ uint8_t kConstStrs[] = "0\0URLENCODED\0JSON\0XML\0MULTIPART\0";
#define CS_ZERO (kConstStrs + 0)
#define CS_URLENCODED (kConstStrs + 2)
#define CS_JSON (kConstStrs + 13)
#define CS_XML (kConstStrs + 18)
#define CS_MULTIPART (kConstStrs + 22)

__device__ inline bool ishex(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
__device__ inline uint8_t hexv(uint8_t c) {
  return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
}
__device__ inline uint8_t x2c(uint8_t a, uint8_t b) { return (uint8_t)((hexv(a) << 4) | hexv(b)); }
__device__ inline uint8_t alower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
__device__ inline bool isalnum_(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}
__device__ inline bool isws(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

__device__ bool eq_bytes(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  if (an != bn) return false;
  for (uint32_t i = 0; i < an; i++)
    if (a[i] != b[i]) return false;
  return true;
}
__device__ bool eq_ascii_ci(const uint8_t* a, uint32_t an, const uint8_t* lowered, uint32_t bn) {
  if (an != bn) return false;
  for (uint32_t i = 0; i < an; i++)
    if (alower(a[i]) != lowered[i]) return false;
  return true;
}
__device__ int64_t find_bytes(const uint8_t* h, uint32_t hn, const uint8_t* nd, uint32_t nn) {
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
__device__ int64_t go_atoi(const uint8_t* s, uint32_t n, bool* ok) {
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
__device__ uint32_t go_itoa(int64_t v, uint8_t* buf) {
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
__device__ inline uint32_t decode_rune(const uint8_t* b, uint32_t n, uint32_t i, uint32_t* w) {
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

__device__ inline uint32_t encode_rune(uint32_t r, uint8_t* o) {
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

// --------------------------------------------------------------- DFA scan
// Sticky-accept DFA over rune classes (rune mode: Go UTF-8 decoding) or
// bytes (phrase automata).  fold: ASCII-lowercase bytes before the lookup.
__device__ bool dfa_match(const DProgram& P, int32_t id, const uint8_t* s, uint32_t n, bool fold) {
  const DDfa d = P.dfas[id];
  const uint16_t* __restrict__ tr = P.trans + d.trans_off;
  const uint8_t* __restrict__ amap = P.u8pool + d.amap_off;
  const uint32_t ncls = d.n_classes;
  uint32_t st = d.start;
  uint32_t i = 0;
  if (d.byte_mode) {
    while (i < n) {
      if (st == d.accept) return true;
      uint8_t c = s[i++];
      if (fold) c = alower(c);
      st = tr[st * ncls + amap[c]];
    }
  } else {
    while (i < n) {
      if (st == d.accept) return true;
      uint8_t c = s[i];
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

// ----------------------------------------------------------- transforms
// Each writes dst (capacity cap) and returns the new length, or -1 on
// overflow.  [upstream coraza internal/transformations/*.go]

__device__ uint32_t lower_rune(const DProgram& P, uint32_t r) {
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
__device__ int64_t t_lowercase(const DProgram& P, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
  bool ascii = true;
  for (uint32_t i = 0; i < n; i++)
    if (s[i] >= 0x80) { ascii = false; break; }
  if (ascii) {
    if (n > cap) return -1;
    for (uint32_t i = 0; i < n; i++) d[i] = alower(s[i]);
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
__device__ int64_t t_urldecode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
__device__ int64_t t_urldecodeuni(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
__device__ uint8_t strtol_byte(const uint8_t* s, uint32_t n, uint32_t base) {
  uint64_t acc = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t v = base == 16 ? hexv(s[i]) : (uint32_t)(s[i] - '0');
    if (acc > ((uint64_t)INT64_MAX - v) / base) return 0xFF;
    acc = acc * base + v;
  }
  return (uint8_t)(acc & 0xFF);
}

// ModSecurity html_entities_decode_inplace (t:htmlEntityDecode)
__device__ int64_t t_htmlentitydecode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
          const uint8_t* x = s + k;
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

__device__ inline bool ws_or_nbsp(uint8_t c) { return isws(c) || c == 0xA0; }

__device__ int64_t t_simple(uint8_t code, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
__device__ inline bool go_isspace(uint32_t r) {
  if (r <= 0xFF) return r == ' ' || (r >= 9 && r <= 13) || r == 0x85 || r == 0xA0;
  return r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 || r == 0x202F ||
         r == 0x205F || r == 0x3000;
}

// Go strings.TrimLeft/TrimRight(unicode.IsSpace)
__device__ int64_t t_trim(uint8_t code, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
__device__ int64_t t_normpath(bool win, const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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

__device__ inline bool isodigit(uint8_t c) { return c >= '0' && c <= '7'; }

// ModSecurity js_decode_nonstrict_inplace (t:jsDecode)
__device__ int64_t t_jsdecode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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
__device__ int64_t t_utf8tounicode(const uint8_t* s, uint32_t n, uint8_t* d, uint32_t cap) {
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

__device__ int64_t apply_transform(const DProgram& P, uint8_t code, const uint8_t* s, uint32_t n, uint8_t* d,
                                   uint32_t cap) {
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
    default: return t_simple(code, s, n, d, cap);
  }
}

// ------------------------------------------------------------ transaction
struct Tx {
  const DProgram* P;
  Field* fields;
  uint32_t nf, cap_f;
  Slot* slots;
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
  const uint32_t* hits;      // phase-A hit words [slot/32][n_req]
  uint32_t n_req, req;
  bool has_post;             // ARGS_POST fields exist (phase-A bits of RF_BODYDEP links void)
  int64_t removed[8][2];
  uint32_t nremoved;
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
  uint8_t itoa_buf[24];
};

__device__ inline uint8_t* tx_alloc(Tx& t, uint32_t n) {
  if (t.nb + n > t.cap_b) {
    t.flags |= GI_REQ_OVERFLOW;
    return nullptr;
  }
  uint8_t* p = t.bytes + t.nb;
  t.nb += n;
  return p;
}

__device__ inline void add_field(Tx& t, uint8_t kind, const uint8_t* k, uint32_t kn, const uint8_t* v, uint32_t vn) {
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
__device__ uint32_t query_unescape(const uint8_t* s, uint32_t n, uint8_t* d) {
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

// coraza internal/url ParseQuery(query, '&') -> fields of `kind`
__device__ void parse_query(Tx& t, const uint8_t* q, uint32_t n, uint8_t kind) {
  uint32_t i = 0;
  while (i < n) {
    uint32_t j = i;
    while (j < n && q[j] != '&') j++;
    if (j > i) {
      uint32_t e = i;
      while (e < j && q[e] != '=') e++;
      const uint8_t* k = q + i;
      uint32_t kn = e - i;
      const uint8_t* v = q + (e < j ? e + 1 : j);
      uint32_t vn = e < j ? j - e - 1 : 0;
      uint8_t* dk = tx_alloc(t, kn + vn);
      if (!dk) return;
      uint32_t dkn = query_unescape(k, kn, dk);
      uint32_t dvn = query_unescape(v, vn, dk + dkn);
      add_field(t, kind, dk, dkn, dk + dkn, dvn);
    }
    i = j + 1;
  }
}

// net/url shouldEscape(c, encodePath)
__device__ inline bool should_escape_path(uint8_t c) {
  if (isalnum_(c)) return false;
  switch (c) {
    case '-': case '_': case '.': case '~': return false;
    case '$': case '&': case '+': case ',': case '/': case ':': case ';': case '=': case '?': case '@':
      return c == '?';
  }
  return true;
}
__device__ inline bool valid_encoded_path_char(uint8_t c) {
  switch (c) {
    case '!': case '$': case '&': case '\'': case '(': case ')': case '*': case '+': case ',': case ';':
    case '=': case ':': case '@': case '[': case ']': case '%':
      return true;
  }
  return !should_escape_path(c);
}

// ProcessURI [upstream corazawaf/transaction.go] + Go net/url Parse/String
__device__ bool process_uri(Tx& t, const uint8_t* uri, uint32_t un) {
  t.single[S_REQUEST_URI_RAW] = {uri, un};
  uint32_t n = un;
  for (uint32_t i = 0; i < un; i++)
    if (uri[i] == '#') { n = i; break; }
  bool ctl = false;
  for (uint32_t i = 0; i < n; i++)
    if (uri[i] < 0x20 || uri[i] == 0x7F) { ctl = true; break; }
  Str path{uri, n}, query{uri, 0};
  if (ctl) {
    t.single[S_REQUEST_URI] = {uri, n};
  } else if (n == 1 && uri[0] == '*') {
    t.single[S_REQUEST_URI] = {uri, 1};
  } else {
    if (n == 0 || uri[0] != '/' || (n >= 2 && uri[1] == '/')) {
      t.flags |= GI_REQ_UNSUPPORTED_URI;
      return false;
    }
    uint32_t nq = 0, q = n;
    for (uint32_t i = 0; i < n; i++)
      if (uri[i] == '?') {
        if (q == n) q = i;
        nq++;
      }
    bool force_q = n > 0 && uri[n - 1] == '?' && nq == 1;
    uint32_t rest_n = q;
    if (force_q) {
      query = {uri + n, 0};
    } else if (q < n) {
      query = {uri + q + 1, n - q - 1};
    }
    // strict unescape(rest, encodePath)
    bool bad = false, has_pct = false;
    for (uint32_t i = 0; i < rest_n; i++)
      if (uri[i] == '%') {
        has_pct = true;
        if (i + 2 >= rest_n || !ishex(uri[i + 1]) || !ishex(uri[i + 2])) { bad = true; break; }
        i += 2;
      }
    if (bad) {
      t.single[S_REQUEST_URI] = {uri, n};
      path = {uri, n};
      query = {uri, 0};
    } else {
      const uint8_t* p = uri;
      uint32_t pn = rest_n;
      if (has_pct) {
        uint8_t* dp = tx_alloc(t, rest_n);
        if (!dp) return false;
        uint32_t o = 0;
        for (uint32_t i = 0; i < rest_n; i++) {
          if (uri[i] == '%') {
            dp[o++] = x2c(uri[i + 1], uri[i + 2]);
            i += 2;
          } else {
            dp[o++] = uri[i];
          }
        }
        p = dp;
        pn = o;
      }
      parse_query(t, query.p, query.n, FK_ARG_GET);
      // EscapedPath: rest if escape(path) == rest or validEncoded(rest), else escape(path)
      bool valid = true;
      for (uint32_t i = 0; i < rest_n; i++)
        if (!valid_encoded_path_char(uri[i])) { valid = false; break; }
      uint32_t esc_len = 0;
      for (uint32_t i = 0; i < pn; i++) esc_len += should_escape_path(p[i]) ? 3 : 1;
      bool same = false;
      if (!valid && esc_len == rest_n) {
        same = true;
        uint32_t o = 0;
        const char* hx = "0123456789ABCDEF";
        for (uint32_t i = 0; i < pn && same; i++) {
          if (should_escape_path(p[i])) {
            same = uri[o] == '%' && uri[o + 1] == hx[p[i] >> 4] && uri[o + 2] == hx[p[i] & 15];
            o += 3;
          } else {
            same = uri[o] == p[i];
            o++;
          }
        }
      }
      if (valid || same) {
        // String() reproduces the fragment-stripped input: rest + "?" + query
        t.single[S_REQUEST_URI] = {uri, n};
      } else {
        const uint32_t tail = (force_q || query.n) ? 1 + query.n : 0;
        uint8_t* o = tx_alloc(t, esc_len + tail);
        if (!o) return false;
        uint32_t k = 0;
        const char* hx = "0123456789ABCDEF";
        for (uint32_t i = 0; i < pn; i++) {
          if (should_escape_path(p[i])) {
            o[k++] = '%';
            o[k++] = hx[p[i] >> 4];
            o[k++] = hx[p[i] & 15];
          } else {
            o[k++] = p[i];
          }
        }
        if (tail) {
          o[k++] = '?';
          for (uint32_t i = 0; i < query.n; i++) o[k++] = query.p[i];
        }
        t.single[S_REQUEST_URI] = {o, k};
      }
      path = {p, pn};
    }
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

__device__ void parse_cookies(Tx& t, const uint8_t* v, uint32_t n) {
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

__device__ inline bool starts_ci(const uint8_t* s, uint32_t n, const char* lit) {
  uint32_t i = 0;
  for (; lit[i]; i++)
    if (i >= n || alower(s[i]) != (uint8_t)lit[i]) return false;
  return true;
}

// ------------------------------------------------------------ TX / macros
__device__ Str slot_str(Tx& t, const Slot& s, uint8_t* buf) {
  if (s.state == 1) return {buf, go_itoa(s.num, buf)};
  if (s.state == 2) return {s.p, s.n};
  return {buf, 0};
}
__device__ int64_t slot_int(const Slot& s, bool* ok) {
  if (s.state == 1) {
    *ok = true;
    return s.num;
  }
  if (s.state == 2) return go_atoi(s.p, s.n, ok);
  *ok = false;
  return 0;
}

// Expand a %{..} template.  *persistent: result points into the program's
// string pool (safe to keep in TX); otherwise into the macro scratch.
__device__ Str expand(Tx& t, int32_t tid, bool* persistent) {
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
      s = slot_str(t, t.slots[p.slot], nb);
    } else if (p.kind == TP_SINGLE) {
      s = t.single[p.single];
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
    for (uint32_t i = 0; i < s.n; i++) t.mt[o + i] = s.p[i];
    o += s.n;
  }
  return {t.mt, o};
}

// setvar [upstream internal/actions/setvar.go]
__device__ void run_setvar(Tx& t, const DAction& a) {
  Slot& sl = t.slots[a.slot];
  if (a.kind == A_SETVAR_DEL) {
    sl.state = 0;
    return;
  }
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
  if (t.ntx + v.n > t.cap_tx) {
    t.flags |= GI_REQ_OVERFLOW;
    return;
  }
  uint8_t* dst = t.txa + t.ntx;
  for (uint32_t i = 0; i < v.n; i++) dst[i] = v.p[i];
  t.ntx += v.n;
  sl.state = 2;
  sl.p = dst;
  sl.n = v.n;
}

__device__ void run_actions(Tx& t, const DRule& R) {
  const DProgram& P = *t.P;
  for (uint32_t k = 0; k < R.act_count; k++) {
    const DAction a = P.acts[R.act_begin + k];
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
__device__ bool contains_word(const uint8_t* v, uint32_t vn, const uint8_t* w, uint32_t wn) {
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

__device__ bool eval_op(Tx& t, const DOp& o, const uint8_t* s, uint32_t n) {
  const DProgram& P = *t.P;
  bool res = false;
  switch (o.kind) {
    case OP_RX:
    case OP_PM:
      res = dfa_match(P, o.dfa, s, n, false);
      break;
    case OP_UNCONDITIONAL:
      res = true;
      break;
    case OP_NOMATCH:
      res = false;
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
        case OP_WITHIN: res = find_bytes(a.p, a.n, s, n) >= 0; break;
      }
    }
  }
  return o.negate ? !res : res;
}

// ------------------------------------------------------------ evaluation
// Apply the rule's transformation chain; returns the value to test.
__device__ Str transform(Tx& t, const DRule& R, const uint8_t* v, uint32_t vn, bool* ok) {
  const DProgram& P = *t.P;
  Str cur{v, vn};
  *ok = true;
  for (uint32_t k = 0; k < R.tchain_len; k++) {
    uint8_t* dst = (cur.p == t.t0) ? t.t1 : t.t0;
    int64_t m = apply_transform(P, P.tchains[R.tchain_off + k], cur.p, cur.n, dst, t.cap_t);
    if (m < 0) {
      t.flags |= GI_REQ_OVERFLOW;
      *ok = false;
      return {dst, 0};
    }
    cur = {dst, (uint32_t)m};
  }
  return cur;
}

__device__ inline bool key_excluded(Tx& t, const DVarRef& vr, const uint8_t* k, uint32_t kn) {
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

__device__ inline bool field_in(uint8_t var, uint32_t kind, bool* names) {
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
  }
  return false;
}

// Test one value: transform, operator, per-match actions.  Returns 1 on match.
__device__ inline uint32_t test_value(Tx& t, const DRule& R, const DOp& o, const uint8_t* v, uint32_t vn) {
  bool ok;
  Str tv = transform(t, R, v, vn, &ok);
  if (!ok) return 0;
  if (eval_op(t, o, tv.p, tv.n)) {
    run_actions(t, R);
    return 1;
  }
  return 0;
}

// Rule.doEvaluate for one link -> number of matched values.
__device__ uint32_t eval_rule(Tx& t, const DRule& R) {
  const DProgram& P = *t.P;
  // phase-A filter: a clear hit bit proves no value matches (exact); a set
  // bit (match or "maybe") falls through to the full evaluation below.
  if (R.hit_slot >= 0 && !((R.flags & RF_BODYDEP) && t.has_post)) {
    const uint32_t w = t.hits[(uint64_t)(R.hit_slot >> 5) * t.n_req + t.req];
    if (!((w >> (R.hit_slot & 31)) & 1u)) return 0;
  }
  if (R.op < 0) {
    run_actions(t, R);
    return 1;
  }
  const DOp o = P.ops[R.op];
  uint32_t nmatch = 0;
  for (uint32_t vi = 0; vi < R.var_count; vi++) {
    const DVarRef vr = P.vars[R.var_begin + vi];
    if (vr.var < S_COUNT) {
      if (vr.count) {
        uint8_t one = '1';
        nmatch += test_value(t, R, o, &one, 1);
      } else {
        Str s = t.single[vr.var];
        nmatch += test_value(t, R, o, s.p, s.n);
      }
      continue;
    }
    if (vr.var == V_TX) {
      uint32_t cnt = 0;
      for (uint32_t sid = 0; sid < P.n_slots; sid++) {
        if (t.slots[sid].state == 0) continue;
        if (vr.key_mode == 1 && (int32_t)sid != vr.slot) continue;
        const uint8_t* nm = P.strpool + P.slot_names[sid * 2];
        uint32_t nn = P.slot_names[sid * 2 + 1];
        if (vr.key_mode == 2 && !dfa_match(P, vr.key_dfa, nm, nn, false)) continue;
        if (key_excluded(t, vr, nm, nn)) continue;
        if (vr.count) {
          cnt++;
          continue;
        }
        Str s = slot_str(t, t.slots[sid], t.itoa_buf);
        nmatch += test_value(t, R, o, s.p, s.n);
      }
      if (vr.count) {
        uint8_t buf[24];
        uint32_t k = go_itoa(cnt, buf);
        nmatch += test_value(t, R, o, buf, k);
      }
      continue;
    }
    uint32_t cnt = 0;
    for (uint32_t f = 0; f < t.nf; f++) {
      const Field fl = t.fields[f];
      bool names;
      if (!field_in(vr.var, fl.kind, &names)) continue;
      if (vr.key_mode == 1) {
        if (vr.ci ? !eq_ascii_ci(fl.k, fl.kn, P.strpool + vr.key_off, vr.key_len)
                  : !eq_bytes(fl.k, fl.kn, P.strpool + vr.key_off, vr.key_len))
          continue;
      } else if (vr.key_mode == 2) {
        if (!dfa_match(P, vr.key_dfa, fl.k, fl.kn, vr.ci != 0)) continue;
      }
      if (vr.exc_count && key_excluded(t, vr, fl.k, fl.kn)) continue;
      if (vr.count) {
        cnt++;
        continue;
      }
      if (names)
        nmatch += test_value(t, R, o, fl.k, fl.kn);
      else
        nmatch += test_value(t, R, o, fl.v, fl.vn);
    }
    if (vr.count) {
      uint8_t buf[24];
      uint32_t k = go_itoa(cnt, buf);
      nmatch += test_value(t, R, o, buf, k);
    }
  }
  return nmatch;
}

__device__ void eval_top(Tx& t, uint32_t ri) {
  const DProgram& P = *t.P;
  const DRule R = P.rules[ri];
  if (eval_rule(t, R) == 0) return;
  for (int32_t ci = R.chain_next; ci >= 0; ci = P.rules[ci].chain_next) {
    const DRule C = P.rules[ci];
    if (eval_rule(t, C) == 0) return;
  }
  if (R.skip_after >= 0) t.skip_after = R.skip_after;
  if (R.skip) t.skip = R.skip;
  if ((R.disruptive == D_DENY || R.disruptive == D_DROP || R.disruptive == D_REDIRECT) && t.engine == ENGINE_ON) {
    t.interrupted = true;
    t.int_rule = R.id;
    t.int_status = R.status;
    t.int_action = R.disruptive == D_DENY ? GI_ACTION_DENY : R.disruptive == D_DROP ? GI_ACTION_DROP
                                                                                     : GI_ACTION_REDIRECT;
    t.int_phase = t.phase;
  }
  if (R.id != 0) {
    if (t.nmatched < t.mcap) t.mout[t.nmatched] = (uint32_t)R.id;
    else t.flags |= GI_REQ_MATCH_TRUNC;
    t.nmatched++;
  }
}

// RuleGroup.Eval [upstream corazawaf/rulegroup.go]
__device__ void eval_phase(Tx& t, uint8_t phase) {
  const DProgram& P = *t.P;
  if (t.engine == ENGINE_OFF) return;
  t.phase = phase;
  for (uint32_t k = 0; k < P.n_top; k++) {
    if (t.interrupted) break;
    if (t.flags & GI_REQ_ERROR_MASK) break;
    const uint32_t ri = P.top[k];
    const DRule& R = P.rules[ri];
    const uint8_t rph = R.phase;
    if (rph != 0 && rph != phase) continue;
    const int32_t id = R.id;
    if (id != 0 && t.nremoved) {
      bool rm = false;
      for (uint32_t j = 0; j < t.nremoved; j++)
        if (t.removed[j][0] <= id && id <= t.removed[j][1]) rm = true;
      if (rm) continue;
    }
    if (t.skip_after >= 0) {
      if (R.marker == t.skip_after) t.skip_after = -1;
      continue;
    }
    if (t.skip > 0) {
      t.skip--;
      continue;
    }
    if (R.flags & RF_MARKER) continue;
    eval_top(t, ri);
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
  uint8_t _pad[7];
  Str single[S_COUNT];
};
static_assert(sizeof(ReqHdr) <= 256, "ReqHdr must fit its 256-byte slot");

struct Region {
  ReqHdr* hdr;
  Field* fields;
  Slot* slots;
  uint8_t *bytes, *t0, *t1, *mt, *txa;
  uint32_t cap_f, cap_b, cap_t, cap_mt;
};

__device__ inline Region region_of(const DProgram& P, const DBatch& B, uint32_t r) {
  const ReqLayout L = B.layout[r];
  uint8_t* base = B.scratch + L.base;
  Region g;
  g.hdr = (ReqHdr*)base;
  uint64_t off = 256;
  g.fields = (Field*)(base + off);
  off += (uint64_t)L.cap_f * sizeof(Field);
  g.slots = (Slot*)(base + off);
  off += ((uint64_t)P.n_slots * sizeof(Slot) + 15) & ~15ull;
  g.bytes = base + off;
  off += (L.cap_b + 15) & ~15u;
  g.t0 = base + off;
  off += (L.cap_t + 15) & ~15u;
  g.t1 = base + off;
  off += (L.cap_t + 15) & ~15u;
  g.mt = base + off;
  off += (L.cap_mt + 15) & ~15u;
  g.txa = base + off;
  g.cap_f = L.cap_f;
  g.cap_b = L.cap_b;
  g.cap_t = L.cap_t;
  g.cap_mt = L.cap_mt;
  return g;
}

__device__ inline void tx_bind(Tx& t, const DProgram& P, const Region& g) {
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
  t.cap_tx = g.cap_mt;
  t.single = g.hdr->single;
}

// ------------------------------------------------ stage 1: k_collect
// ProcessURI + AddRequestHeader* for one request per thread.  Fields are
// grouped by kind so each scan group walks only its own range.
__global__ void __launch_bounds__(256) k_collect(DProgram P, DBatch B) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B.n_req) return;
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
  uint8_t* ln = tx_alloc(t, method.n + uri.n + proto.n + 2);
  if (ln) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < method.n; i++) ln[k++] = method.p[i];
    ln[k++] = ' ';
    for (uint32_t i = 0; i < uri.n; i++) ln[k++] = uri.p[i];
    ln[k++] = ' ';
    for (uint32_t i = 0; i < proto.n; i++) ln[k++] = proto.p[i];
    t.single[S_REQUEST_LINE] = {ln, k};
  }
  const bool ok = process_uri(t, uri.p, uri.n);
  const uint32_t n_get = t.nf;
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
  H->nb = t.nb;
  H->n_get = (uint16_t)n_get;
  H->n_hdr = (uint16_t)n_hdr;
  H->n_ck = (uint16_t)(t.nf - n_get - n_hdr);
  H->flags = t.flags | ((t.nf > 0xFFFF) ? GI_REQ_OVERFLOW : 0);
  H->body_proc = t.body_proc;
}

// ------------------------------------------------ stage 2: k_match (phase A)
// Persistent kernel over units (job, tile of 256 requests), job-major.  A
// workgroup copies the job's automaton image (<= 64 KB) into LDS once per job
// change, then each thread walks one request: the stream's values are key-
// filtered, transformed once and run through every automaton of the job whose
// admitted patterns intersect the value's filter-pass mask.

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

// Bit k of the result: pattern k of the automaton matches somewhere in s.
// Single (sticky) automata return bit 0 only.
__device__ __forceinline__ uint64_t jdfa_scan(const DProgram& P, const DDfa& d, const uint16_t* __restrict__ tr,
                                              const uint8_t* __restrict__ amap, const uint8_t* __restrict__ combo,
                                              const uint8_t* __restrict__ s, uint32_t n) {
  const uint32_t ncls = d.n_classes;
  uint32_t st = d.start;
  uint32_t i = 0;
  if (!d.multi) {
    while (i < n) {
      if (st == d.accept) return 1;
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
      st = tr[st * ncls + cls];
    }
    return P.u8pool[d.endacc_off + st] != 0 ? 1ull : 0ull;
  }
  const uint64_t* __restrict__ acc = P.u64pool + d.acc_off;
  uint64_t m = 0;
  while (i < n) {
    const uint8_t c = s[i];
    uint32_t cls;
    if (c < 0x80) {
      cls = amap[c];
      i++;
    } else {
      uint32_t w;
      const uint32_t rr = decode_rune(s, n, i, &w);
      i += w;
      cls = rune_class(P, d, rr);
    }
    const uint16_t tv = tr[st * ncls + cls];
    if (tv & 0x8000) m |= acc[(uint64_t)st * 5 + combo[cls]];
    st = tv & 0x7FFF;
  }
  return m | acc[(uint64_t)st * 5 + 4];
}

__device__ inline bool validate_op(uint8_t kind, const uint32_t* bits, const uint8_t* s, uint32_t n) {
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

__device__ inline void set_hit(const DBatch& B, uint32_t slot, uint32_t r) {
  atomicOr(&B.hits[(uint64_t)(slot >> 5) * B.n_req + r], 1u << (slot & 31));
}

// Key filter of a rule target (selector + exclusions), as field_in() applies it.
__device__ inline bool filter_ok(const DProgram& P, const DFilter& F, const Field& f) {
  if (F.key_mode == 1) {
    if (F.ci ? !eq_ascii_ci(f.k, f.kn, P.strpool + F.key_off, F.key_len)
             : !eq_bytes(f.k, f.kn, P.strpool + F.key_off, F.key_len))
      return false;
  } else if (F.key_mode == 2) {
    if (!dfa_match(P, F.key_dfa, f.k, f.kn, F.ci != 0)) return false;
  }
  for (uint32_t e = 0; e < F.exc_count; e++) {
    const DExc x = P.excs[F.exc_begin + e];
    if (x.dfa >= 0) {
      if (dfa_match(P, x.dfa, f.k, f.kn, true)) return false;
    } else if (eq_ascii_ci(f.k, f.kn, P.strpool + x.off, x.len)) {
      return false;
    }
  }
  return true;
}

// transform (chain) + match one value against the job; hit bits are emitted
// per value (matches are rare); "maybe" (every admitted pattern) on overflow.
__device__ void match_value(const DProgram& P, const DBatch& B, uint32_t r, const DStream& S, const DJob& J,
                            const uint8_t* img, uint32_t fm, const uint8_t* v, uint32_t vn, uint8_t* s0,
                            uint8_t* s1) {
  const uint8_t* cur = v;
  uint32_t cn = vn;
  bool maybe = false;
  bool ready = false;
  for (uint32_t q = 0; q < J.jdfa_count + J.val_count; q++) {
    uint64_t allowed = 0;
    DJobDfa jd;
    if (q < J.jdfa_count) {
      jd = P.jdfas[J.jdfa_begin + q];
      for (uint32_t f = fm; f; f &= f - 1) allowed |= P.u64pool[jd.fmask_off + (__ffs(f) - 1)];
      if (!allowed) continue;
    } else if (!(fm & P.svals[J.val_begin + q - J.jdfa_count].fmask)) {
      continue;
    }
    if (!ready) {
      ready = true;
      for (uint32_t k = 0; k < S.tchain_len; k++) {
        uint8_t* dst = (cur == s0) ? s1 : s0;
        int64_t m = apply_transform(P, P.tchains[S.tchain_off + k], cur, cn, dst, B.tcap);
        if (m < 0) {
          maybe = true;
          break;
        }
        cur = dst;
        cn = (uint32_t)m;
      }
    }
    if (q < J.jdfa_count) {
      uint64_t m = allowed;
      if (!maybe) {
        const DDfa d = P.dfas[jd.dfa];
        uint64_t x;
        if (jd.lds_trans >= 0) {
          x = jdfa_scan(P, d, (const uint16_t*)(img + jd.lds_trans), img + jd.lds_amap,
                        img + (jd.lds_combo >= 0 ? jd.lds_combo : 0), cur, cn);
        } else {
          x = jdfa_scan(P, d, P.trans + d.trans_off, P.u8pool + d.amap_off, P.u8pool + d.combo_off, cur, cn);
        }
        m &= x ^ jd.neg_mask;
      }
      while (m) {
        const int k = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        set_hit(B, P.pats[jd.pat_begin + k].slot, r);
      }
    } else {
      const DScanVal& sv = P.svals[J.val_begin + q - J.jdfa_count];
      if (maybe || (validate_op(sv.kind, sv.bits, cur, cn) != (sv.negate != 0))) set_hit(B, sv.slot, r);
    }
  }
}

__global__ void __launch_bounds__(256) k_match(DProgram P, DBatch B, uint32_t n_tiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* s0 = B.tscratch + (uint64_t)tid * 2ull * B.tcap;
  uint8_t* s1 = s0 + B.tcap;
  const uint64_t n_units = (uint64_t)P.n_jobs * n_tiles;
  uint32_t loaded = 0xFFFFFFFFu;
  for (uint64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    const uint32_t j = (uint32_t)(u / n_tiles);
    const uint32_t tile = (uint32_t)(u - (uint64_t)j * n_tiles);
    const DJob J = P.jobs[j];
    if (j != loaded) {  // block-uniform
      __syncthreads();
      const uint4* src = (const uint4*)(P.images + J.img_off);
      for (uint32_t k = threadIdx.x; k < J.img_bytes / 16; k += blockDim.x) ((uint4*)img)[k] = src[k];
      __syncthreads();
      loaded = j;
    }
    const uint32_t r = tile * 256 + threadIdx.x;
    if (r >= B.n_req) continue;
    const uint8_t* base = B.scratch + B.layout[r].base;
    const ReqHdr* H = (const ReqHdr*)base;
    if (H->flags & GI_REQ_ERROR_MASK) continue;
    const DStream S = P.streams[J.stream];
    for (uint32_t k = 0; k < S.filt_count; k++) {
      const uint8_t sg = P.filters[S.filt_begin + k].single;
      if (sg == GI_NO_SINGLE) continue;
      const Str v = H->single[sg];
      match_value(P, B, r, S, J, img, 1u << k, v.p, v.n, s0, s1);
    }
    if (!S.kind_mask) continue;
    const Field* F = (const Field*)(base + 256);
    const uint32_t n_get = H->n_get, n_hdr = H->n_hdr, n_ck = H->n_ck;
    for (int kind = FK_ARG_GET; kind <= FK_COOKIE; kind++) {
      if (!((S.kind_mask >> kind) & 1)) continue;
      uint32_t b = 0, e = 0;
      if (kind == FK_ARG_GET) { b = 0; e = n_get; }
      else if (kind == FK_HEADER) { b = n_get; e = n_get + n_hdr; }
      else if (kind == FK_COOKIE) { b = n_get + n_hdr; e = n_get + n_hdr + n_ck; }
      else continue;
      for (uint32_t i = b; i < e; i++) {
        const Field f = F[i];
        uint32_t fv = 0, fk = 0;
        for (uint32_t k = 0; k < S.filt_count; k++) {
          const DFilter Fl = P.filters[S.filt_begin + k];
          if (Fl.single != GI_NO_SINGLE || !((Fl.kind_mask >> kind) & 1)) continue;
          if (filter_ok(P, Fl, f)) {
            if (Fl.names) fk |= 1u << k;
            else fv |= 1u << k;
          }
        }
        if (fv) match_value(P, B, r, S, J, img, fv, f.v, f.vn, s0, s1);
        if (fk) match_value(P, B, r, S, J, img, fk, f.k, f.kn, s0, s1);
      }
    }
  }
}

// ------------------------------------------------ stage 3: k_eval (phase B)
// RuleGroup.Eval(1) -> ProcessRequestBody -> RuleGroup.Eval(2) per request,
// skipping every phase-A rule whose hit bit is clear.
__global__ void __launch_bounds__(128) k_eval(DProgram P, DBatch B) {
  __shared__ unsigned long long red[6];
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x < 6) red[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long my[6] = {0, 0, 0, 0, 0, 0};
  if (r < B.n_req) {
    const gi_request rq = B.reqs[r];
    Region g = region_of(P, B, r);
    ReqHdr* H = g.hdr;
    Tx t;
    tx_bind(t, P, g);
    t.hits = B.hits;
    t.n_req = B.n_req;
    t.req = r;
    t.has_post = false;
    t.nf = H->nf;
    t.nb = H->nb;
    t.flags = H->flags;
    t.body_proc = H->body_proc;
    t.ntx = 0;
    t.nremoved = 0;
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
    t.mcap = B.mcap;
    for (uint32_t s = 0; s < P.n_slots; s++) t.slots[s].state = 0;
    const uint8_t* D = B.data;
    uint64_t scanned = (uint64_t)rq.method.len + rq.uri.len + rq.proto.len + rq.body.len;
    for (uint32_t h = 0; h < rq.hdr_count; h++) {
      const gi_header hd = B.headers[rq.hdr_begin + h];
      scanned += hd.name.len + hd.value.len;
    }
    if (!(t.flags & GI_REQ_ERROR_MASK)) {
      eval_phase(t, 1);
      if (!t.interrupted && t.engine != ENGINE_OFF && !(t.flags & GI_REQ_ERROR_MASK)) {
        const uint32_t bn = rq.body.len;
        if (t.body_access && bn > 0) {
          if (bn > P.body_limit) {
            t.flags |= GI_REQ_BODY_LIMIT;
          } else {
            uint8_t* lb = tx_alloc(t, 24);
            if (lb) t.single[S_REQUEST_BODY_LENGTH] = {lb, go_itoa((int64_t)bn, lb)};
            if (t.force_body && t.body_proc == BP_NONE) {
              t.body_proc = BP_URLENCODED;
              t.single[S_REQBODY_PROCESSOR] = {CS_URLENCODED, 10};
            }
            if (t.body_proc == BP_URLENCODED) {
              t.single[S_REQUEST_BODY] = {D + rq.body.off, bn};
              const uint32_t nf0 = t.nf;
              parse_query(t, D + rq.body.off, bn, FK_ARG_POST);
              t.has_post = t.nf > nf0;
            } else if (t.body_proc != BP_NONE) {
              t.flags |= GI_REQ_UNSUPPORTED_BODY;
            }
          }
        }
        if (!(t.flags & GI_REQ_ERROR_MASK)) eval_phase(t, 2);
      }
    }
    gi_verdict v;
    v.rule_id = t.interrupted ? t.int_rule : 0;
    v.status = t.interrupted ? t.int_status : 0;
    v.action = t.interrupted ? t.int_action : 0;
    v.phase = t.interrupted ? t.int_phase : 0;
    v.flags = t.flags;
    v.match_cnt = t.nmatched;
    for (uint32_t e = 0; e < GI_MAX_EXPORTS; e++) {
      int64_t x = 0;
      if (e < P.n_exports && P.exports[e] >= 0) {
        bool okk;
        x = slot_int(t.slots[P.exports[e]], &okk);
        if (!okk) x = 0;
      }
      v.tx_export[e] = x;
    }
    B.verdicts[r] = v;
    my[0] = 1;
    my[1] = t.interrupted ? 1 : 0;
    my[2] = t.nmatched ? 1 : 0;
    my[3] = (t.flags & GI_REQ_ERROR_MASK) ? 1 : 0;
    my[4] = scanned;
    my[5] = t.nmatched;
  }
  for (int c = 0; c < 6; c++) {
    unsigned long long x = my[c];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[c], x);
  }
  __syncthreads();
  if (threadIdx.x < 6) atomicAdd(&B.tally[threadIdx.x], red[threadIdx.x]);
}

uint32_t scan_resident_threads(uint32_t lds_bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, dev);
  int per_cu = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_match, 256, lds_bytes);
  if (per_cu < 1) per_cu = 1;
  return (uint32_t)prop.multiProcessorCount * (uint32_t)per_cu * 256u;
}

void launch_pipeline(const DProgram& P, const DBatch& B, uint32_t scan_threads, hipStream_t stream,
                     hipEvent_t* ev) {
  if (!B.n_req) return;
  const uint32_t cb = (B.n_req + 255) / 256;
  hipLaunchKernelGGL(k_collect, dim3(cb), dim3(256), 0, stream, P, B);
  if (ev) (void)hipEventRecord(ev[0], stream);
  const uint32_t n_tiles = (B.n_req + 255) / 256;
  const uint64_t units = (uint64_t)P.n_jobs * n_tiles;
  if (units) {
    uint64_t blocks = units;
    const uint64_t maxb = scan_threads / 256;
    if (blocks > maxb) blocks = maxb;
    hipLaunchKernelGGL(k_match, dim3((uint32_t)blocks), dim3(256), P.max_img_bytes, stream, P, B, n_tiles);
  }
  if (ev) (void)hipEventRecord(ev[1], stream);
  hipLaunchKernelGGL(k_eval, dim3((B.n_req + 127) / 128), dim3(128), 0, stream, P, B);
}

}  // namespace gi
