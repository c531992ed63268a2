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

  bool parse_alt(int flags, int* out) {
    std::vector<int> branches;
    for (;;) {
      int b;
      if (!parse_concat(flags, &b)) return false;
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

  bool parse_concat(int flags, int* out) {
    std::vector<int> items;
    last_rep = false;
    while (!eof()) {
      uint32_t c = peek();
      if (c == '|' || c == ')') break;
      if (c == '*' || c == '+' || c == '?') {
        if (items.empty()) return fail("missing argument to repetition operator");
        i++;
        int lo = c == '+' ? 1 : 0, hi = c == '?' ? 1 : -1;
        if (!apply_repeat(&items, lo, hi, flags)) return false;
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
          if (!apply_repeat(&items, lo, hi, flags)) return false;
          continue;
        }
        i++;
        items.push_back(lit('{', flags));
        last_rep = false;
        continue;
      }
      last_rep = false;
      int atom = -1;
      if (!parse_atom(&flags, &atom)) return false;
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

// ------------------------------------------------------------------- NFA
enum InstOp : uint8_t { I_CLASS, I_SPLIT, I_EMPTY, I_MATCH, I_NOP };
struct Inst {
  InstOp op;
  int out = -1, out1 = -1;
  uint8_t assert_kind = 0;
  int cset = -1;  // index of class bitset
};
struct Frag {
  int start;
  std::vector<std::pair<int, int>> outs;  // (inst, which)
};

struct NfaBuilder {
  const Regex& re;
  std::vector<Inst> prog;
  const std::vector<int>& node_cset;  // node index -> cset id (N_CLASS)
  size_t cap;
  bool overflow = false;

  NfaBuilder(const Regex& r, const std::vector<int>& nc, size_t c) : re(r), node_cset(nc), cap(c) {}

  int emit(Inst in) {
    if (prog.size() >= cap) overflow = true;
    prog.push_back(in);
    return (int)prog.size() - 1;
  }
  void patch(const std::vector<std::pair<int, int>>& outs, int to) {
    for (auto& o : outs) {
      if (o.second == 0)
        prog[o.first].out = to;
      else
        prog[o.first].out1 = to;
    }
  }
  Frag nop() {
    Inst in;
    in.op = I_NOP;
    int k = emit(in);
    return {k, {{k, 0}}};
  }
  Frag cat(Frag a, Frag b) {
    patch(a.outs, b.start);
    return {a.start, std::move(b.outs)};
  }
  Frag star(Frag x) {
    Inst in;
    in.op = I_SPLIT;
    in.out = x.start;
    int s = emit(in);
    patch(x.outs, s);
    return {s, {{s, 1}}};
  }
  Frag plus(Frag x) {
    Inst in;
    in.op = I_SPLIT;
    in.out = x.start;
    int s = emit(in);
    patch(x.outs, s);
    return {x.start, {{s, 1}}};
  }
  Frag quest(Frag x) {
    Inst in;
    in.op = I_SPLIT;
    in.out = x.start;
    int s = emit(in);
    x.outs.push_back({s, 1});
    return {s, std::move(x.outs)};
  }
  Frag compile(int id) {
    if (overflow) return nop();
    const ReNode& n = re.nodes[id];
    switch (n.kind) {
      case N_CLASS: {
        Inst in;
        in.op = I_CLASS;
        in.cset = node_cset[id];
        int k = emit(in);
        return {k, {{k, 0}}};
      }
      case N_EMPTY:
        return nop();
      case N_ASSERT: {
        Inst in;
        in.op = I_EMPTY;
        in.assert_kind = n.assert_kind;
        int k = emit(in);
        return {k, {{k, 0}}};
      }
      case N_CAPTURE:
        return compile(n.kids[0]);
      case N_CAT: {
        Frag f = compile(n.kids[0]);
        for (size_t k = 1; k < n.kids.size(); k++) f = cat(std::move(f), compile(n.kids[k]));
        return f;
      }
      case N_ALT: {
        // right-nested splits
        Frag f = compile(n.kids.back());
        for (int k = (int)n.kids.size() - 2; k >= 0; k--) {
          Frag a = compile(n.kids[k]);
          Inst in;
          in.op = I_SPLIT;
          in.out = a.start;
          in.out1 = f.start;
          int s = emit(in);
          std::vector<std::pair<int, int>> outs = std::move(a.outs);
          outs.insert(outs.end(), f.outs.begin(), f.outs.end());
          f = {s, std::move(outs)};
        }
        return f;
      }
      case N_REPEAT: {
        int sub = n.kids[0];
        if (n.max == -1) {
          if (n.min == 0) return star(compile(sub));
          Frag f = compile(sub);
          for (int k = 1; k < n.min; k++) f = cat(std::move(f), compile(sub));
          // x{min,}: last copy loops
          Frag last = plus(compile(sub));
          if (n.min == 1) return last;
          return cat(std::move(f), std::move(last));
        }
        if (n.max == 0) return nop();
        Frag f;
        bool have = false;
        for (int k = 0; k < n.min; k++) {
          Frag c = compile(sub);
          f = have ? cat(std::move(f), std::move(c)) : std::move(c);
          have = true;
        }
        // (max-min) nested optionals: (x(x(x)?)?)?
        if (n.max > n.min) {
          Frag opt = quest(compile(sub));
          for (int k = n.min + 1; k < n.max; k++) {
            Frag c = compile(sub);
            Frag inner = cat(std::move(c), std::move(opt));
            opt = quest(std::move(inner));
          }
          f = have ? cat(std::move(f), std::move(opt)) : std::move(opt);
          have = true;
        }
        return f;
      }
    }
    return nop();
  }
};

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

// ------------------------------------------------------ DFA minimisation
static void minimize(Dfa* d) {
  const uint32_t n = d->n_states, k = d->n_classes;
  std::vector<uint32_t> block(n);
  for (uint32_t s = 0; s < n; s++) block[s] = s == d->accept ? 0 : (d->end_accept[s] ? 1 : 2);
  uint32_t nblocks = 0;
  for (;;) {
    std::unordered_map<std::string, uint32_t> sig;
    std::vector<uint32_t> nb(n);
    std::string key;
    for (uint32_t s = 0; s < n; s++) {
      key.assign((const char*)&block[s], 4);
      for (uint32_t c = 0; c < k; c++) key.append((const char*)&block[d->trans[s * k + c]], 4);
      auto it = sig.find(key);
      if (it == sig.end()) it = sig.emplace(key, (uint32_t)sig.size()).first;
      nb[s] = it->second;
    }
    uint32_t cnt = (uint32_t)sig.size();
    block.swap(nb);
    if (cnt == nblocks) break;
    nblocks = cnt;
  }
  // renumber: start first, accept second
  std::vector<int> newid(nblocks, -1);
  uint32_t next = 0;
  newid[block[d->start]] = next++;
  if (newid[block[d->accept]] < 0) newid[block[d->accept]] = next++;
  for (uint32_t s = 0; s < n; s++)
    if (newid[block[s]] < 0) newid[block[s]] = next++;
  std::vector<uint16_t> tr((size_t)nblocks * k);
  std::vector<uint8_t> ea(nblocks);
  for (uint32_t s = 0; s < n; s++) {
    uint32_t b = newid[block[s]];
    ea[b] = d->end_accept[s];
    for (uint32_t c = 0; c < k; c++) tr[(size_t)b * k + c] = (uint16_t)newid[block[d->trans[(size_t)s * k + c]]];
  }
  d->start = newid[block[d->start]];
  d->accept = newid[block[d->accept]];
  d->n_states = nblocks;
  d->trans.swap(tr);
  d->end_accept.swap(ea);
}

// ------------------------------------------------------- public: regex DFA
bool build_regex_dfa(const Regex& re, Dfa* out, std::string* err, uint32_t state_cap) {
  *out = Dfa();
  // 1. rune-class partition over every set in the AST + word chars + '\n'
  std::vector<const RuneSet*> sets;
  std::vector<int> node_set(re.nodes.size(), -1);
  RuneSet nl = {{'\n', '\n'}};
  sets.push_back(&kPerlW);
  sets.push_back(&nl);
  {
    std::unordered_map<std::string, int> uniq;
    for (size_t i = 0; i < re.nodes.size(); i++) {
      if (re.nodes[i].kind != N_CLASS) continue;
      std::string key((const char*)re.nodes[i].set.data(), re.nodes[i].set.size() * sizeof(RuneRange));
      auto it = uniq.find(key);
      if (it == uniq.end()) {
        sets.push_back(&re.nodes[i].set);
        it = uniq.emplace(key, (int)sets.size() - 1).first;
      }
      node_set[i] = it->second;
    }
  }
  std::vector<uint32_t> bounds = {0, kMaxRune + 1};
  for (auto* s : sets)
    for (auto& r : *s) {
      bounds.push_back(r.lo);
      bounds.push_back(r.hi + 1);
    }
  for (uint32_t c = 0; c <= 0x80; c++) bounds.push_back(c);  // every ASCII byte is an interval
  std::sort(bounds.begin(), bounds.end());
  bounds.erase(std::unique(bounds.begin(), bounds.end()), bounds.end());
  const size_t nsets = sets.size();
  std::vector<size_t> cursor(nsets, 0);
  std::unordered_map<std::string, uint32_t> sigmap;
  std::vector<std::vector<uint8_t>> class_members;  // class -> membership per set
  std::vector<uint32_t> interval_class;
  for (size_t b = 0; b + 1 < bounds.size(); b++) {
    uint32_t lo = bounds[b];
    std::string sig(nsets, '\0');
    for (size_t si = 0; si < nsets; si++) {
      const RuneSet& rs = *sets[si];
      size_t& cu = cursor[si];
      while (cu < rs.size() && rs[cu].hi < lo) cu++;
      sig[si] = (cu < rs.size() && rs[cu].lo <= lo) ? 1 : 0;
    }
    auto it = sigmap.find(sig);
    if (it == sigmap.end()) {
      it = sigmap.emplace(sig, (uint32_t)class_members.size()).first;
      class_members.emplace_back(sig.begin(), sig.end());
    }
    interval_class.push_back(it->second);
  }
  const uint32_t ncls = (uint32_t)class_members.size();
  if (ncls > 255) {
    *err = "regex needs more than 255 rune classes";
    return false;
  }
  out->n_classes = ncls;
  out->amap.assign(128, 0);
  for (size_t b = 0; b + 1 < bounds.size(); b++) {
    uint32_t lo = bounds[b], hi = bounds[b + 1] - 1;
    if (lo < 0x80) {
      for (uint32_t c = lo; c <= hi && c < 0x80; c++) out->amap[c] = (uint8_t)interval_class[b];
    } else {
      uint32_t cl = interval_class[b];
      size_t m = out->nranges.size();
      if (m >= 3 && out->nranges[m - 1] == cl && out->nranges[m - 2] + 1 == lo)
        out->nranges[m - 2] = hi;
      else {
        out->nranges.push_back(lo);
        out->nranges.push_back(hi);
        out->nranges.push_back(cl);
      }
    }
  }
  const uint32_t cls_nl = out->amap['\n'];
  std::vector<uint8_t> cls_word(ncls);
  for (uint32_t c = 0; c < ncls; c++) cls_word[c] = class_members[c][0];
  // class bitsets per unique set
  const size_t words = (ncls + 63) / 64;
  std::vector<std::vector<uint64_t>> set_bits(nsets, std::vector<uint64_t>(words, 0));
  for (uint32_t c = 0; c < ncls; c++)
    for (size_t si = 0; si < nsets; si++)
      if (class_members[c][si]) set_bits[si][c >> 6] |= 1ull << (c & 63);

  // 2. Thompson NFA
  NfaBuilder nb(re, node_set, 200000);
  Frag f = nb.compile(re.root);
  Inst m;
  m.op = I_MATCH;
  int mpc = nb.emit(m);
  nb.patch(f.outs, mpc);
  if (nb.overflow) {
    *err = "regex too large";
    return false;
  }
  const std::vector<Inst>& prog = nb.prog;
  const int start_pc = f.start;
  uint8_t used = 0;
  for (auto& in : prog)
    if (in.op == I_EMPTY) used |= in.assert_kind;
  const bool need_bol = used & (AS_BOT | AS_BOL);
  const bool need_word = used & (AS_WB | AS_NWB);

  // 3. subset construction (RE2-style flags, sticky accept, unanchored)
  enum { FL_BOT = 1, FL_NL = 2, FL_WORD = 4 };
  struct St {
    std::vector<int> kernel;
    uint8_t flags;
  };
  std::vector<St> states;
  std::unordered_map<std::string, uint32_t> smap;
  std::vector<uint32_t> mark(prog.size(), 0);
  uint32_t gen = 0;
  auto key_of = [](const std::vector<int>& k, uint8_t fl) {
    std::string s((const char*)k.data(), k.size() * sizeof(int));
    s.push_back((char)fl);
    return s;
  };
  auto intern = [&](std::vector<int> k, uint8_t fl) -> uint32_t {
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    if (!need_bol) fl &= ~(FL_BOT | FL_NL);
    if (!need_word) fl &= ~FL_WORD;
    std::string key = key_of(k, fl);
    auto it = smap.find(key);
    if (it != smap.end()) return it->second;
    uint32_t id = (uint32_t)states.size();
    states.push_back({std::move(k), fl});
    smap.emplace(std::move(key), id);
    return id;
  };
  const uint32_t ACCEPT = 0;
  states.push_back({{}, 0});  // state 0 = ACCEPT (kernel ignored)
  smap.emplace(std::string("ACCEPT"), 0);
  uint32_t start = intern({start_pc}, FL_BOT);
  std::vector<int> stack, classes_pcs;
  // closure with the given satisfied-assertion set; returns true on MATCH
  auto closure = [&](const std::vector<int>& kernel, uint8_t cond, std::vector<int>* cpcs) -> bool {
    gen++;
    cpcs->clear();
    stack.assign(kernel.begin(), kernel.end());
    bool matched = false;
    while (!stack.empty()) {
      int pc = stack.back();
      stack.pop_back();
      if (pc < 0 || mark[pc] == gen) continue;
      mark[pc] = gen;
      const Inst& in = prog[pc];
      switch (in.op) {
        case I_MATCH: matched = true; break;
        case I_CLASS: cpcs->push_back(pc); break;
        case I_NOP: stack.push_back(in.out); break;
        case I_SPLIT: stack.push_back(in.out1); stack.push_back(in.out); break;
        case I_EMPTY:
          if ((in.assert_kind & cond) == in.assert_kind) stack.push_back(in.out);
          break;
      }
    }
    return matched;
  };
  std::vector<uint16_t> trans;
  std::vector<uint8_t> end_acc;
  std::vector<int> nk;
  for (uint32_t sid = 1; sid < states.size(); sid++) {
    if (states.size() > state_cap) {
      *err = "regex DFA exceeds state cap";
      return false;
    }
    const std::vector<int> kernel = states[sid].kernel;
    const uint8_t fl = states[sid].flags;
    trans.resize((size_t)(sid + 1) * ncls, 0);
    end_acc.resize(sid + 1, 0);
    const bool bot = fl & FL_BOT, prevnl = fl & FL_NL, prevw = fl & FL_WORD;
    uint8_t base = 0;
    if (bot) base |= AS_BOT;
    if (bot || prevnl) base |= AS_BOL;
    // end of text
    {
      uint8_t cond = base | AS_EOT | AS_EOL | (prevw ? AS_WB : AS_NWB);
      std::vector<int> tmp;
      end_acc[sid] = closure(kernel, cond, &tmp) ? 1 : 0;
    }
    // cache closures by (is_nl, is_word)
    std::vector<int> cl[4];
    bool clm[4];
    bool have[4] = {false, false, false, false};
    for (uint32_t c = 0; c < ncls; c++) {
      const bool isnl = c == cls_nl, isw = cls_word[c];
      int slot = (isnl ? 1 : 0) | (isw ? 2 : 0);
      if (!have[slot]) {
        uint8_t cond = base | (isnl ? AS_EOL : 0) | ((prevw != isw) ? AS_WB : AS_NWB);
        clm[slot] = closure(kernel, cond, &cl[slot]);
        have[slot] = true;
      }
      if (clm[slot]) {
        trans[(size_t)sid * ncls + c] = ACCEPT;
        continue;
      }
      nk.clear();
      nk.push_back(start_pc);
      for (int pc : cl[slot]) {
        const Inst& in = prog[pc];
        if (set_bits[in.cset][c >> 6] >> (c & 63) & 1) nk.push_back(in.out);
      }
      uint8_t nfl = (isnl ? FL_NL : 0) | (isw ? FL_WORD : 0);
      uint32_t t = intern(nk, nfl);
      if (t > 65535) {
        *err = "regex DFA exceeds state cap";
        return false;
      }
      trans[(size_t)sid * ncls + c] = (uint16_t)t;
    }
  }
  const uint32_t n = (uint32_t)states.size();
  trans.resize((size_t)n * ncls, 0);
  end_acc.resize(n, 0);
  for (uint32_t c = 0; c < ncls; c++) trans[c] = ACCEPT;  // state 0 absorbing
  end_acc[0] = 1;
  out->n_states = n;
  out->start = start;
  out->accept = ACCEPT;
  out->trans.swap(trans);
  out->end_accept.swap(end_acc);
  minimize(out);
  return true;
}

// ----------------------------------------------------- public: phrase DFA
bool build_phrase_dfa(const std::vector<std::string>& phrases, bool fold_ascii, Dfa* out,
                      std::string* err, uint32_t state_cap) {
  *out = Dfa();
  out->byte_mode = true;
  auto fb = [&](uint8_t c) -> uint8_t { return (fold_ascii && c >= 'A' && c <= 'Z') ? c + 32 : c; };
  // byte classes: every byte used in a phrase gets its own class; others = 0
  std::vector<int> bcls(256, -1);
  uint32_t ncls = 1;
  for (auto& p : phrases)
    for (uint8_t c : p) {
      uint8_t f = fb(c);
      if (bcls[f] < 0) bcls[f] = ncls++;
    }
  out->amap.assign(256, 0);
  for (int b = 0; b < 256; b++) {
    int f = fb((uint8_t)b);
    out->amap[b] = bcls[f] < 0 ? 0 : (uint8_t)bcls[f];
  }
  if (ncls > 256) {
    *err = "too many byte classes";
    return false;
  }
  // trie
  struct TNode {
    std::vector<int> next;
    int fail = 0;
    bool out = false;
  };
  std::vector<TNode> t(1);
  t[0].next.assign(ncls, -1);
  bool empty_phrase = false;
  for (auto& p : phrases) {
    if (p.empty()) empty_phrase = true;
    int s = 0;
    for (uint8_t c : p) {
      int k = out->amap[c];
      if (t[s].next[k] < 0) {
        t[s].next[k] = (int)t.size();
        TNode nn;
        nn.next.assign(ncls, -1);
        t.push_back(std::move(nn));
      }
      s = t[s].next[k];
    }
    t[s].out = true;
    if (t.size() + 2 > state_cap) {
      *err = "phrase automaton exceeds state cap";
      return false;
    }
  }
  // BFS failure links -> full goto
  std::queue<int> q;
  for (uint32_t k = 0; k < ncls; k++) {
    int c = t[0].next[k];
    if (c < 0) t[0].next[k] = 0;
    else {
      t[c].fail = 0;
      q.push(c);
    }
  }
  while (!q.empty()) {
    int s = q.front();
    q.pop();
    t[s].out = t[s].out || t[t[s].fail].out;
    for (uint32_t k = 0; k < ncls; k++) {
      int c = t[s].next[k];
      if (c < 0) {
        t[s].next[k] = t[t[s].fail].next[k];
      } else {
        t[c].fail = t[t[s].fail].next[k];
        q.push(c);
      }
    }
  }
  // DFA: state 0 = ACCEPT, trie node i -> i+1
  const uint32_t n = (uint32_t)t.size() + 1;
  out->n_classes = ncls;
  out->n_states = n;
  out->accept = 0;
  out->start = (empty_phrase || t[0].out) ? 0 : 1;
  out->trans.assign((size_t)n * ncls, 0);
  out->end_accept.assign(n, 0);
  out->end_accept[0] = 1;
  for (size_t i = 0; i < t.size(); i++)
    for (uint32_t k = 0; k < ncls; k++) {
      int d = t[i].next[k];
      out->trans[(i + 1) * ncls + k] = t[d].out ? 0 : (uint16_t)(d + 1);
    }
  minimize(out);
  return true;
}

bool dfa_host_match(const Dfa& d, const uint8_t* s, size_t n) {
  uint32_t st = d.start;
  size_t i = 0;
  while (i < n) {
    if (st == d.accept) return true;
    uint32_t cls;
    if (d.byte_mode) {
      cls = d.amap[s[i]];
      i++;
    } else if (s[i] < 0x80) {
      cls = d.amap[s[i]];
      i++;
    } else {
      int w;
      uint32_t r = go_decode_rune(s, n, i, &w);
      i += w;
      cls = 0;
      for (size_t k = 0; k + 2 < d.nranges.size(); k += 3) {
        if (r >= d.nranges[k] && r <= d.nranges[k + 1]) {
          cls = d.nranges[k + 2];
          break;
        }
      }
    }
    st = d.trans[(size_t)st * d.n_classes + cls];
  }
  return d.end_accept[st] != 0;
}

}  // namespace gi
