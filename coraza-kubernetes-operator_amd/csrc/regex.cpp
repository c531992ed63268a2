// RE2-syntax parser + rune-class DFA construction (host side of @rx / @pm).
// See regex.h for the contract and the reference anchors.
#include "regex.h"

#include <algorithm>
#include <queue>
#include <unordered_map>

#include "unicode_tables.h"

namespace gi {
namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr int kMaxRepeat = 1000;
enum { F_I = 1, F_M = 2, F_S = 4, F_U = 8 };

// ---------------------------------------------------------------- rune sets
void clean(RuneSet* rs) {
  std::sort(rs->begin(), rs->end(), [](const RuneRange& a, const RuneRange& b) {
    return a.lo < b.lo || (a.lo == b.lo && a.hi < b.hi);
  });
  RuneSet out;
  for (const auto& r : *rs) {
    if (!out.empty() && r.lo <= out.back().hi + 1) {
      if (r.hi > out.back().hi) out.back().hi = r.hi;
    } else {
      out.push_back(r);
    }
  }
  *rs = std::move(out);
}

RuneSet negate(RuneSet rs) {
  clean(&rs);
  RuneSet out;
  uint32_t next = 0;
  for (const auto& r : rs) {
    if (r.lo > next) out.push_back({next, r.lo - 1});
    next = r.hi + 1;
  }
  if (next <= kMaxRune) out.push_back({next, kMaxRune});
  return out;
}

// unicode.SimpleFold orbit closure of every rune in the set.
RuneSet fold(RuneSet rs) {
  RuneSet add;
  for (const auto& r : rs) {
    const uint32_t(*b)[2] = std::lower_bound(
        kFoldPairs, kFoldPairs + GI_N_FOLD_PAIRS, r.lo,
        [](const uint32_t(&p)[2], uint32_t v) { return p[0] < v; });
    for (; b != kFoldPairs + GI_N_FOLD_PAIRS && (*b)[0] <= r.hi; ++b) add.push_back({(*b)[1], (*b)[1]});
  }
  rs.insert(rs.end(), add.begin(), add.end());
  clean(&rs);
  return rs;
}

const RuneSet kPerlD = {{0x30, 0x39}};
const RuneSet kPerlS = {{0x09, 0x0A}, {0x0C, 0x0D}, {0x20, 0x20}};
const RuneSet kPerlW = {{0x30, 0x39}, {0x41, 0x5A}, {0x5F, 0x5F}, {0x61, 0x7A}};

bool posix_class(const std::string& name, RuneSet* out) {
  static const std::vector<std::pair<const char*, RuneSet>> tab = {
      {"alnum", {{0x30, 0x39}, {0x41, 0x5A}, {0x61, 0x7A}}},
      {"alpha", {{0x41, 0x5A}, {0x61, 0x7A}}},
      {"ascii", {{0x00, 0x7F}}},
      {"blank", {{0x09, 0x09}, {0x20, 0x20}}},
      {"cntrl", {{0x00, 0x1F}, {0x7F, 0x7F}}},
      {"digit", {{0x30, 0x39}}},
      {"graph", {{0x21, 0x7E}}},
      {"lower", {{0x61, 0x7A}}},
      {"print", {{0x20, 0x7E}}},
      {"punct", {{0x21, 0x2F}, {0x3A, 0x40}, {0x5B, 0x60}, {0x7B, 0x7E}}},
      {"space", {{0x09, 0x0D}, {0x20, 0x20}}},
      {"upper", {{0x41, 0x5A}}},
      {"word", {{0x30, 0x39}, {0x41, 0x5A}, {0x5F, 0x5F}, {0x61, 0x7A}}},
      {"xdigit", {{0x30, 0x39}, {0x41, 0x46}, {0x61, 0x66}}},
  };
  for (const auto& e : tab)
    if (name == e.first) {
      *out = e.second;
      return true;
    }
  return false;
}

bool is_alnum(uint32_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}
int unhex(uint32_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// ------------------------------------------------------------------ parser
struct Parser {
  std::vector<uint32_t> s;
  size_t i = 0;
  Regex* re;
  std::string err;
  bool last_rep = false;

  bool fail(const char* m) {
    if (err.empty()) err = m;
    return false;
  }
  bool eof() const { return i >= s.size(); }
  uint32_t peek(size_t k = 0) const { return i + k < s.size() ? s[i + k] : 0xFFFFFFFFu; }

  int add(ReNode n) {
    re->nodes.push_back(std::move(n));
    return (int)re->nodes.size() - 1;
  }
  int lit(uint32_t r, int flags) {
    ReNode n;
    n.kind = N_CLASS;
    n.set = {{r, r}};
    if (flags & F_I) n.set = fold(n.set);
    return add(std::move(n));
  }
  int cls(RuneSet rs) {
    ReNode n;
    n.kind = N_CLASS;
    clean(&rs);
    n.set = std::move(rs);
    return add(std::move(n));
  }
  int empty() {
    ReNode n;
    n.kind = N_EMPTY;
    return add(std::move(n));
  }
  int assertion(uint8_t k) {
    ReNode n;
    n.kind = N_ASSERT;
    n.assert_kind = k;
    return add(std::move(n));
  }

  RuneSet perl_group(uint32_t c, int flags) {
    RuneSet rs = (c == 'd' || c == 'D') ? kPerlD : (c == 's' || c == 'S') ? kPerlS : kPerlW;
    if (flags & F_I) rs = fold(rs);
    if (c == 'D' || c == 'S' || c == 'W') rs = negate(rs);
    return rs;
  }

  // Go parseEscape; i points at '\\'.
  bool escape(uint32_t* r) {
    i++;
    if (eof()) return fail("trailing backslash at end of expression");
    uint32_t c = s[i++];
    if (c < 0x80 && !is_alnum(c)) {
      *r = c;
      return true;
    }
    if (c >= '1' && c <= '7') {
      if (eof() || s[i] < '0' || s[i] > '7') return fail("invalid escape sequence");
    }
    if (c >= '0' && c <= '7') {
      uint32_t v = c - '0';
      for (int k = 0; k < 2; k++) {
        if (!eof() && s[i] >= '0' && s[i] <= '7') {
          v = v * 8 + (s[i] - '0');
          i++;
        } else {
          break;
        }
      }
      *r = v;
      return true;
    }
    if (c == 'x') {
      if (eof()) return fail("invalid escape sequence");
      if (s[i] == '{') {
        i++;
        uint32_t v = 0;
        int nhex = 0;
        for (;;) {
          if (eof()) return fail("invalid escape sequence");
          uint32_t d = s[i++];
          if (d == '}') break;
          int h = unhex(d);
          if (h < 0) return fail("invalid escape sequence");
          v = v * 16 + h;
          if (v > kMaxRune) return fail("invalid escape sequence");
          nhex++;
        }
        if (nhex == 0) return fail("invalid escape sequence");
        *r = v;
        return true;
      }
      if (i + 1 >= s.size()) return fail("invalid escape sequence");
      int x = unhex(s[i]), y = unhex(s[i + 1]);
      if (x < 0 || y < 0) return fail("invalid escape sequence");
      i += 2;
      *r = x * 16 + y;
      return true;
    }
    switch (c) {
      case 'a': *r = 7; return true;
      case 'f': *r = 12; return true;
      case 'n': *r = 10; return true;
      case 'r': *r = 13; return true;
      case 't': *r = 9; return true;
      case 'v': *r = 11; return true;
    }
    return fail("invalid escape sequence");
  }

  bool class_char(uint32_t* r) {
    if (peek() == '\\') return escape(r);
    *r = s[i++];
    return true;
  }

  bool parse_class(int flags, int* out) {
    i++;  // [
    bool neg = false;
    if (peek() == '^') {
      neg = true;
      i++;
    }
    RuneSet rs;
    bool first = true;
    for (;;) {
      if (eof()) return fail("missing closing ]");
      uint32_t c = peek();
      if (c == ']' && !first) {
        i++;
        break;
      }
      first = false;
      if (c == '[' && peek(1) == ':') {
        size_t j = i + 2;
        while (j + 1 < s.size() && !(s[j] == ':' && s[j + 1] == ']')) j++;
        if (j + 1 < s.size()) {
          std::string name;
          for (size_t k = i + 2; k < j; k++) name.push_back((char)s[k]);
          bool pneg = !name.empty() && name[0] == '^';
          if (pneg) name = name.substr(1);
          RuneSet g;
          if (!posix_class(name, &g)) return fail("invalid character class range");
          if (flags & F_I) g = fold(g);
          if (pneg) g = negate(g);
          rs.insert(rs.end(), g.begin(), g.end());
          i = j + 2;
          continue;
        }
      }
      if (c == '\\') {
        uint32_t k = peek(1);
        if (k == 'd' || k == 's' || k == 'w' || k == 'D' || k == 'S' || k == 'W') {
          RuneSet g = perl_group(k, flags);
          rs.insert(rs.end(), g.begin(), g.end());
          i += 2;
          continue;
        }
        if (k == 'p' || k == 'P') return fail("unsupported Unicode class escape");
      }
      uint32_t lo, hi;
      if (!class_char(&lo)) return false;
      hi = lo;
      if (peek() == '-' && i + 1 < s.size() && s[i + 1] != ']') {
        i++;
        if (!class_char(&hi)) return false;
        if (hi < lo) return fail("invalid character class range");
      }
      RuneSet one = {{lo, hi}};
      if (flags & F_I) one = fold(one);
      rs.insert(rs.end(), one.begin(), one.end());
    }
    clean(&rs);
    if (neg) rs = negate(rs);
    *out = cls(std::move(rs));
    return true;
  }

  // Go parseRepeat / parseInt ({n}, {n,}, {n,m}; no leading zeros).
  bool try_brace(int* lo, int* hi, size_t* after) {
    size_t j = i + 1;
    auto parse_int = [&](int* v) -> bool {
      if (j >= s.size() || s[j] < '0' || s[j] > '9') return false;
      if (j + 1 < s.size() && s[j] == '0' && s[j + 1] >= '0' && s[j + 1] <= '9') return false;
      long n = 0;
      while (j < s.size() && s[j] >= '0' && s[j] <= '9') {
        if (n >= 100000000) n = 100000000;
        else n = n * 10 + (s[j] - '0');
        j++;
      }
      *v = n >= 100000000 ? -1 : (int)n;
      return true;
    };
    if (!parse_int(lo)) return false;
    if (j >= s.size()) return false;
    if (s[j] != ',') {
      *hi = *lo;
    } else {
      j++;
      if (j >= s.size()) return false;
      if (s[j] == '}') {
        *hi = -1;
      } else {
        if (!parse_int(hi)) return false;
        if (*hi < 0) *lo = -1;
      }
    }
    if (j >= s.size() || s[j] != '}') return false;
    *after = j + 1;
    return true;
  }

  bool apply_repeat(std::vector<int>* items, int lo, int hi, int flags) {
    bool greedy = true;
    if (peek() == '?') {
      i++;
      greedy = false;
    }
    if (last_rep) return fail("invalid nested repetition operator");
    if (flags & F_U) greedy = !greedy;
    ReNode n;
    n.kind = N_REPEAT;
    n.kids = {items->back()};
    n.min = lo;
    n.max = hi;
    n.greedy = greedy;
    items->back() = add(std::move(n));
    last_rep = true;
    return true;
  }

  // A flag group (?i) persists to the end of the enclosing group, across '|'
  // (Go regexp/syntax): the branches share one flags variable.
  bool parse_alt(int flags, int* out) {
    std::vector<int> branches;
    for (;;) {
      int b;
      if (!parse_concat(&flags, &b)) return false;
      branches.push_back(b);
      if (peek() == '|') {
        i++;
        continue;
      }
      break;
    }
    if (branches.size() == 1) {
      *out = branches[0];
      return true;
    }
    ReNode n;
    n.kind = N_ALT;
    n.kids = std::move(branches);
    *out = add(std::move(n));
    return true;
  }

  bool parse_concat(int* flags, int* out) {
    std::vector<int> items;
    last_rep = false;
    while (!eof()) {
      uint32_t c = peek();
      if (c == '|' || c == ')') break;
      if (c == '*' || c == '+' || c == '?') {
        if (items.empty()) return fail("missing argument to repetition operator");
        i++;
        int lo = c == '+' ? 1 : 0, hi = c == '?' ? 1 : -1;
        if (!apply_repeat(&items, lo, hi, *flags)) return false;
        continue;
      }
      if (c == '{') {
        int lo, hi;
        size_t after;
        if (try_brace(&lo, &hi, &after)) {
          if (lo < 0 || lo > kMaxRepeat || hi > kMaxRepeat || (hi >= 0 && lo > hi))
            return fail("invalid repeat count");
          if (items.empty()) return fail("missing argument to repetition operator");
          i = after;
          if (!apply_repeat(&items, lo, hi, *flags)) return false;
          continue;
        }
        i++;
        items.push_back(lit('{', *flags));
        last_rep = false;
        continue;
      }
      last_rep = false;
      int atom = -1;
      if (!parse_atom(flags, &atom)) return false;
      if (atom >= 0) items.push_back(atom);
    }
    if (items.empty()) {
      *out = empty();
    } else if (items.size() == 1) {
      *out = items[0];
    } else {
      ReNode n;
      n.kind = N_CAT;
      n.kids = std::move(items);
      *out = add(std::move(n));
    }
    return true;
  }

  bool parse_group(int* flags, int* out) {
    i++;  // (
    if (peek() == '?') {
      // named capture (?P<name>..) / (?<name>..)
      bool pnamed = peek(1) == 'P' && peek(2) == '<';
      bool anamed = peek(1) == '<' && peek(2) != '=' && peek(2) != '!';
      if (pnamed || anamed) {
        size_t j = i + (pnamed ? 3 : 2);
        size_t st = j;
        while (j < s.size() && s[j] != '>') {
          if (!(is_alnum(s[j]) || s[j] == '_')) return fail("invalid named capture");
          j++;
        }
        if (j >= s.size() || j == st) return fail("invalid named capture");
        i = j + 1;
        int idx = ++re->ncap;
        int inner;
        if (!parse_alt(*flags, &inner)) return false;
        if (peek() != ')') return fail("missing closing )");
        i++;
        ReNode n;
        n.kind = N_CAPTURE;
        n.cap = idx;
        n.kids = {inner};
        *out = add(std::move(n));
        return true;
      }
      size_t j = i + 1;
      int sign = 1;
      bool saw = false;
      int nf = *flags;
      for (;;) {
        if (j >= s.size()) return fail("missing closing )");
        uint32_t ch = s[j];
        int bit = ch == 'i' ? F_I : ch == 'm' ? F_M : ch == 's' ? F_S : ch == 'U' ? F_U : 0;
        if (bit) {
          nf = sign > 0 ? (nf | bit) : (nf & ~bit);
          saw = true;
          j++;
          continue;
        }
        if (ch == '-') {
          if (sign < 0) return fail("invalid or unsupported Perl syntax");
          sign = -1;
          saw = false;
          j++;
          continue;
        }
        if (ch == ':' || ch == ')') {
          if (sign < 0 && !saw) return fail("invalid or unsupported Perl syntax");
          if (ch == ')' && j == i + 1) return fail("invalid or unsupported Perl syntax");
          break;
        }
        return fail("invalid or unsupported Perl syntax");
      }
      if (s[j] == ')') {
        i = j + 1;
        *flags = nf;  // applies to the rest of the enclosing group
        *out = -1;
        return true;
      }
      i = j + 1;
      int inner;
      if (!parse_alt(nf, &inner)) return false;
      if (peek() != ')') return fail("missing closing )");
      i++;
      *out = inner;
      return true;
    }
    int idx = ++re->ncap;
    int inner;
    if (!parse_alt(*flags, &inner)) return false;
    if (peek() != ')') return fail("missing closing )");
    i++;
    ReNode n;
    n.kind = N_CAPTURE;
    n.cap = idx;
    n.kids = {inner};
    *out = add(std::move(n));
    return true;
  }

  bool parse_atom(int* flags, int* out) {
    uint32_t c = peek();
    if (c == '(') {
      bool ok = parse_group(flags, out);
      last_rep = false;
      return ok;
    }
    if (c == '[') return parse_class(*flags, out);
    if (c == '.') {
      i++;
      if (*flags & F_S)
        *out = cls({{0, kMaxRune}});
      else
        *out = cls({{0, 9}, {11, kMaxRune}});
      return true;
    }
    if (c == '^') {
      i++;
      *out = assertion((*flags & F_M) ? AS_BOL : AS_BOT);
      return true;
    }
    if (c == '$') {
      i++;
      *out = assertion((*flags & F_M) ? AS_EOL : AS_EOT);
      return true;
    }
    if (c == '\\') {
      if (i + 1 >= s.size()) return fail("trailing backslash at end of expression");
      uint32_t k = s[i + 1];
      switch (k) {
        case 'A': i += 2; *out = assertion(AS_BOT); return true;
        case 'z': i += 2; *out = assertion(AS_EOT); return true;
        case 'b': i += 2; *out = assertion(AS_WB); return true;
        case 'B': i += 2; *out = assertion(AS_NWB); return true;
        case 'Q': {
          i += 2;
          std::vector<int> lits;
          while (i < s.size()) {
            if (s[i] == '\\' && i + 1 < s.size() && s[i + 1] == 'E') {
              i += 2;
              break;
            }
            lits.push_back(lit(s[i], *flags));
            i++;
          }
          if (lits.empty()) {
            *out = -1;
          } else if (lits.size() == 1) {
            *out = lits[0];
          } else {
            ReNode n;
            n.kind = N_CAT;
            n.kids = std::move(lits);
            *out = add(std::move(n));
          }
          return true;
        }
        case 'd': case 's': case 'w': case 'D': case 'S': case 'W':
          i += 2;
          *out = cls(perl_group(k, *flags));
          return true;
        case 'p': case 'P':
          return fail("unsupported Unicode class escape");
        case 'C':
          return fail("invalid escape sequence");
      }
      uint32_t r;
      if (!escape(&r)) return false;
      *out = lit(r, *flags);
      return true;
    }
    i++;
    *out = lit(c, *flags);
    return true;
  }
};

bool utf8_to_runes(const std::string& p, std::vector<uint32_t>* out) {
  const uint8_t* b = (const uint8_t*)p.data();
  size_t n = p.size(), i = 0;
  while (i < n) {
    if (b[i] < 0x80) {
      out->push_back(b[i]);
      i++;
      continue;
    }
    int w;
    uint32_t r = go_decode_rune(b, n, i, &w);
    if (r == 0xFFFD && w == 1) return false;
    out->push_back(r);
    i += w;
  }
  return true;
}

}  // namespace

// ------------------------------------------------------------ public: parse
bool re_parse(const std::string& pattern, Regex* out, std::string* err) {
  *out = Regex();
  Parser p;
  p.re = out;
  if (!utf8_to_runes(pattern, &p.s)) {
    *err = "invalid UTF-8";
    return false;
  }
  int root;
  int flags = 0;
  if (!p.parse_alt(flags, &root)) {
    *err = p.err;
    return false;
  }
  if (!p.eof()) {
    *err = "unexpected )";
    return false;
  }
  out->root = root;
  return true;
}

uint32_t go_decode_rune(const uint8_t* b, size_t n, size_t i, int* w) {
  uint8_t c0 = b[i];
  if (c0 < 0x80) {
    *w = 1;
    return c0;
  }
  int need;
  uint8_t lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) need = 1;
  else if (c0 == 0xE0) { need = 2; lo = 0xA0; }
  else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) need = 2;
  else if (c0 == 0xED) { need = 2; hi = 0x9F; }
  else if (c0 == 0xF0) { need = 3; lo = 0x90; }
  else if (c0 >= 0xF1 && c0 <= 0xF3) need = 3;
  else if (c0 == 0xF4) { need = 3; hi = 0x8F; }
  else { *w = 1; return 0xFFFD; }
  if (n - i < (size_t)need + 1) { *w = 1; return 0xFFFD; }
  uint8_t c1 = b[i + 1];
  if (c1 < lo || c1 > hi) { *w = 1; return 0xFFFD; }
  for (int k = 2; k <= need; k++)
    if (b[i + k] < 0x80 || b[i + k] > 0xBF) { *w = 1; return 0xFFFD; }
  uint32_t r;
  if (need == 1) r = ((c0 & 0x1F) << 6) | (c1 & 0x3F);
  else if (need == 2) r = ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (b[i + 2] & 0x3F);
  else r = ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((b[i + 2] & 0x3F) << 6) | (b[i + 3] & 0x3F);
  *w = need + 1;
  return r;
}

}  // namespace gi
