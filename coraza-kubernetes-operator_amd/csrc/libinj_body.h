// libinjection restated for the device: the definitions (no include guard,
// no namespace).  libinj.h includes them once in namespace gi for every
// caller; kernels.hip includes them a second time in namespace gi::lid for
// k_detect alone, so that copy is compiled for k_detect's occupancy target
// instead of the register budget of the other callers (k_eval / k_stream /
// k_long).  See libinj.h for the algorithm notes.

// ------------------------------------------------------------- SQLi ----
enum : uint8_t {
  LI_FLAG_QUOTE_NONE = 1, LI_FLAG_QUOTE_SINGLE = 2, LI_FLAG_QUOTE_DOUBLE = 4,
  LI_FLAG_SQL_ANSI = 8, LI_FLAG_SQL_MYSQL = 16,
};
#define LI_TOKEN_SIZE 32
#define LI_MAX_TOKENS 5

struct LiTok {
  const uint8_t* p;  // value bytes (the input, or the keyword pool after a merge)
  uint16_t len;      // <= LI_TOKEN_SIZE - 1 (st_assign truncation)
  uint8_t type;      // libinjection token type character, 0 = none
  uint8_t sopen, sclose;
  uint8_t _pad[3];
};

// Keyword tables the lookups read: the __constant__ arrays of libinj_words.h,
// or k_detect's LDS copies of them (li_tables_const / k_detect).
struct LiTables {
  const uint32_t* words;  // kLiWords
  const uint8_t* pool;    // kLiPool
  const uint16_t* hash;   // kLiHash
};

// LI_LDS_TABLES (k_detect's copy): an expression for the keyword tables in
// LDS; the state then carries no table pointers (168 B instead of 200 B)
struct LiSqli {
  const uint8_t* s;
  uint32_t slen, flags, pos, cur;
  uint32_t ddx, hash, ntok;
#ifndef LI_LDS_TABLES
  LiTables T;
#endif
  LiTok tv[8];
#ifndef LI_LDS_TABLES
  uint32_t _pad[2];  // 200 B = 50 dwords: k_detect's per-lane LDS states hit ~2-way, not 16-way, bank conflicts
#endif
};
#undef LI_T
#ifdef LI_LDS_TABLES
#define LI_T(S) LI_LDS_TABLES
#else
#define LI_T(S) ((S).T)
#endif

GI_HD __forceinline__ LiTables li_tables_const() { return LiTables{kLiWords, kLiPool, kLiHash}; }

GI_HD __forceinline__ uint8_t li_up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// byte i of the lookup key: a, or a + ' ' + b (syntax_merge_words), upper-cased
GI_HD __forceinline__ uint8_t li_key_at(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t i) {
  if (i < an) return li_up(a[i]);
  if (i == an) return ' ';
  return li_up(b[i - an - 1]);
}

// bsearch_keyword_type restated as a hash probe: the index of the word equal
// to the upper-cased key (a, or a + ' ' + b), -1 if none.  FNV-1a over the
// upper-cased bytes into an open-addressing table (tools/gen_libinj_tables.py).
GI_HD __forceinline__ int li_find(const LiTables& T, const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn,
                                    bool two) {
  const uint32_t kn = two ? an + 1 + bn : an;
  if (kn == 0 || kn >= LI_TOKEN_SIZE) return -1;
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < kn; i++) {
    const uint8_t c = li_key_at(a, an, b, i);
    if (c == 0) return -1;  // cstrcasecmp never equates a NUL
    h = (h ^ c) * 16777619u;
  }
  for (uint32_t slot = h & (LI_HASH_SIZE - 1);; slot = (slot + 1) & (LI_HASH_SIZE - 1)) {
    const uint32_t idx = T.hash[slot];
    if (!idx) return -1;
    const uint32_t e = T.words[idx - 1];
    if (((e >> 16) & 0xFFu) != kn) continue;
    const uint8_t* w = T.pool + (e & 0xFFFFu);
    bool eq = true;
    for (uint32_t i = 0; i < kn && eq; i++) eq = w[i] == li_key_at(a, an, b, i);
    if (eq) return (int)(idx - 1);
  }
}
GI_HD __forceinline__ uint8_t li_lookup(const LiTables& T, const uint8_t* a, uint32_t an) {
  const int i = li_find(T, a, an, nullptr, 0, false);
  return i < 0 ? (uint8_t)0 : (uint8_t)(T.words[i] >> 24);
}

// cstrcasecmp(lit, tok, tok.len) == 0 (lit upper case, no NUL)
GI_HD __forceinline__ bool li_tok_is(const LiTok& t, const char* lit) {
  uint32_t i = 0;
  for (; lit[i]; i++)
    if (i >= t.len || li_up(t.p[i]) != (uint8_t)lit[i]) return false;
  return i == t.len;
}

GI_HD __forceinline__ bool li_white(uint8_t c) {  // char_is_white: " \t\n\v\f\r\240\000"
  return c == ' ' || (c >= 9 && c <= 13) || c == 0xA0 || c == 0;
}

GI_HD __forceinline__ bool li_word_stop(uint8_t c) {
  // parse_word's strlencspn set " []{}<>:\\?=@!#~+-*/&|^%(),';\t\n\v\f\r\"\240\000"
  switch (c) {
    case ' ': case '[': case ']': case '{': case '}': case '<': case '>': case ':': case '\\': case '?':
    case '=': case '@': case '!': case '#': case '~': case '+': case '-': case '*': case '/': case '&':
    case '|': case '^': case '%': case '(': case ')': case ',': case '\'': case ';': case '\t': case '\n':
    case '\v': case '\f': case '\r': case '"': case 0xA0: case 0: return true;
  }
  return false;
}

GI_HD __forceinline__ bool li_var_stop(uint8_t c) {
  // parse_var's set " <>:\\?=@!#~+-*/&|^%(),';\t\n\v\f\r'`\""
  switch (c) {
    case ' ': case '<': case '>': case ':': case '\\': case '?': case '=': case '@': case '!': case '#':
    case '~': case '+': case '-': case '*': case '/': case '&': case '|': case '^': case '%': case '(':
    case ')': case ',': case '\'': case ';': case '\t': case '\n': case '\v': case '\f': case '\r':
    case '`': case '"': return true;
  }
  return false;
}

GI_HD __forceinline__ bool li_isdigit(uint8_t c) { return c >= '0' && c <= '9'; }
GI_HD __forceinline__ bool li_ishex(uint8_t c) {
  return li_isdigit(c) || (c >= 'A' && c <= 'F') || (c >= 'a' && c <= 'f');
}

// memchr2: first i in [b, e - 1) with s[i] == c0 && s[i + 1] == c1; a c0
// not followed by c1 skips two bytes, as the C loop does.  -1 if none.
GI_HD int64_t li_memchr2(const uint8_t* s, uint32_t b, uint32_t e, uint8_t c0, uint8_t c1) {
  if (e < b + 2) return -1;
  uint32_t cur = b;
  const uint32_t last = e - 1;
  while (cur < last) {
    if (s[cur] == c0) {
      if (s[cur + 1] == c1) return cur;
      cur += 2;
    } else {
      cur += 1;
    }
  }
  return -1;
}

GI_HD __forceinline__ int64_t li_memchr(const uint8_t* s, uint32_t b, uint32_t e, uint8_t c) {
  for (uint32_t i = b; i < e; i++)
    if (s[i] == c) return i;
  return -1;
}

GI_HD __forceinline__ void li_assign(LiTok& t, uint8_t type, const uint8_t* p, uint32_t len) {
  t.type = type;
  t.p = p;
  t.len = (uint16_t)(len < LI_TOKEN_SIZE - 1 ? len : LI_TOKEN_SIZE - 1);
}
GI_HD __forceinline__ void li_clear(LiTok& t) {
  t.p = nullptr;
  t.len = 0;
  t.type = 0;
  t.sopen = t.sclose = 0;
}

// parse_string_core: string at pos (first quote skipped when offset > 0)
GI_HD uint32_t li_string_core(const uint8_t* s, uint32_t slen, uint32_t pos, LiTok& st, uint8_t delim,
                                   uint32_t offset) {
  const uint32_t start = pos + offset;
  int64_t q = li_memchr(s, start, slen, delim);
  st.sopen = offset > 0 ? delim : 0;
  while (true) {
    if (q < 0) {
      li_assign(st, 's', s + start, slen - start);
      st.sclose = 0;
      return slen;
    }
    int64_t j = q - 1;  // is_backslash_escaped
    while (j >= (int64_t)start && s[j] == '\\') j--;
    if ((q - 1 - j) & 1) {
      q = li_memchr(s, (uint32_t)q + 1, slen, delim);
      continue;
    }
    if ((uint32_t)q + 1 < slen && s[q + 1] == s[q]) {  // is_double_delim_escaped
      q = li_memchr(s, (uint32_t)q + 2 > slen ? slen : (uint32_t)q + 2, slen, delim);
      continue;
    }
    li_assign(st, 's', s + start, (uint32_t)q - start);
    st.sclose = delim;
    return (uint32_t)q + 1;
  }
}

enum : uint8_t {
  LP_WHITE, LP_OP1, LP_OP2, LP_OTHER, LP_CHAR, LP_STRING, LP_HASH, LP_MONEY, LP_DASH, LP_NUMBER,
  LP_SLASH, LP_VAR, LP_WORD, LP_BSTRING, LP_ESTRING, LP_NQSTRING, LP_QSTRING, LP_USTRING,
  LP_XSTRING, LP_BWORD, LP_BACKSLASH, LP_TICK,
};

// char_parse_map
GI_HD __forceinline__ uint8_t li_parser(uint8_t c) {
  if (c <= 32 || c == 127 || c == 160) return LP_WHITE;
  if (li_isdigit(c) || c == '.') return LP_NUMBER;
  switch (c) {
    case '!': case '&': case '*': case ':': case '<': case '=': case '>': case '|': return LP_OP2;
    case '%': case '+': case '^': case '~': return LP_OP1;
    case '"': case '\'': return LP_STRING;
    case '#': return LP_HASH;
    case '$': return LP_MONEY;
    case '(': case ')': case ',': case ';': case '{': case '}': return LP_CHAR;
    case '-': return LP_DASH;
    case '/': return LP_SLASH;
    case '?': case ']': return LP_OTHER;
    case '@': return LP_VAR;
    case 'B': case 'b': return LP_BSTRING;
    case 'E': case 'e': return LP_ESTRING;
    case 'N': case 'n': return LP_NQSTRING;
    case 'Q': case 'q': return LP_QSTRING;
    case 'U': case 'u': return LP_USTRING;
    case 'X': case 'x': return LP_XSTRING;
    case '[': return LP_BWORD;
    case '\\': return LP_BACKSLASH;
    case '`': return LP_TICK;
  }
  return LP_WORD;
}

GI_HD __forceinline__ uint32_t li_parse_word(LiSqli& S, LiTok& c, uint32_t pos) {
  const uint8_t* s = S.s;
  uint32_t e = pos;
  while (e < S.slen && !li_word_stop(s[e])) e++;
  const uint32_t wlen = e - pos;
  li_assign(c, 'n', s + pos, wlen);
  for (uint32_t i = 0; i < c.len; i++) {
    const uint8_t d = c.p[i];
    if (d == '.' || d == '`') {
      const uint8_t ch = li_lookup(LI_T(S), c.p, i);
      if (ch != 0 && ch != 'n') {
        li_clear(c);
        li_assign(c, ch, s + pos, i);
        return pos + i;
      }
    }
  }
  if (wlen < LI_TOKEN_SIZE) {
    const uint8_t ch = li_lookup(LI_T(S), c.p, wlen);
    c.type = ch ? ch : 'n';
  }
  return pos + wlen;
}

GI_HD uint32_t li_parse_eol_comment(LiSqli& S, LiTok& c, uint32_t pos) {
  const int64_t e = li_memchr(S.s, pos, S.slen, '\n');
  if (e < 0) {
    li_assign(c, 'c', S.s + pos, S.slen - pos);
    return S.slen;
  }
  li_assign(c, 'c', S.s + pos, (uint32_t)e - pos);
  return (uint32_t)e + 1;
}

GI_HD uint32_t li_parse_qstring_core(LiSqli& S, LiTok& c, uint32_t p0, uint32_t offset) {
  const uint8_t* s = S.s;
  const uint32_t slen = S.slen, pos = p0 + offset;
  if (pos >= slen || (s[pos] != 'q' && s[pos] != 'Q') || pos + 2 >= slen || s[pos + 1] != '\'')
    return li_parse_word(S, c, p0);
  uint8_t ch = s[pos + 2];
  if (ch < 33 || ch > 127) return li_parse_word(S, c, p0);
  ch = ch == '(' ? ')' : ch == '[' ? ']' : ch == '{' ? '}' : ch == '<' ? '>' : ch;
  const int64_t e = li_memchr2(s, pos + 3, slen, ch, '\'');
  c.sopen = 'q';
  if (e < 0) {
    li_assign(c, 's', s + pos + 3, slen - pos - 3);
    c.sclose = 0;
    return slen;
  }
  li_assign(c, 's', s + pos + 3, (uint32_t)e - pos - 3);
  c.sclose = 'q';
  return (uint32_t)e + 2;
}

GI_HD uint32_t li_parse_estring(LiSqli& S, LiTok& c, uint32_t pos) {
  if (pos + 2 >= S.slen || S.s[pos + 1] != '\'') return li_parse_word(S, c, pos);
  return li_string_core(S.s, S.slen, pos, c, '\'', 2);
}

GI_HD uint32_t li_parse_tick(LiSqli& S, LiTok& c, uint32_t pos) {
  const uint32_t np = li_string_core(S.s, S.slen, pos, c, '`', 1);
  const uint8_t ch = li_lookup(LI_T(S), c.p, c.len);
  c.type = ch == 'f' ? 'f' : 'n';
  return np;
}

GI_HD __forceinline__ uint32_t li_parse_money(LiSqli& S, LiTok& c, uint32_t pos) {
  const uint8_t* s = S.s;
  const uint32_t slen = S.slen;
  if (pos + 1 == slen) {
    li_assign(c, 'n', s + pos, 1);
    return slen;
  }
  uint32_t xlen = 0;
  while (pos + 1 + xlen < slen && (li_isdigit(s[pos + 1 + xlen]) || s[pos + 1 + xlen] == '.' || s[pos + 1 + xlen] == ','))
    xlen++;
  if (xlen == 0) {
    if (s[pos + 1] == '$') {
      const int64_t e = li_memchr2(s, pos + 2, slen, '$', '$');
      c.sopen = '$';
      if (e < 0) {
        li_assign(c, 's', s + pos + 2, slen - (pos + 2));
        c.sclose = 0;
        return slen;
      }
      li_assign(c, 's', s + pos + 2, (uint32_t)e - (pos + 2));
      c.sclose = '$';
      return (uint32_t)e + 2;
    }
    while (pos + 1 + xlen < slen &&
           ((s[pos + 1 + xlen] >= 'a' && s[pos + 1 + xlen] <= 'z') || (s[pos + 1 + xlen] >= 'A' && s[pos + 1 + xlen] <= 'Z')))
      xlen++;
    if (xlen == 0 || pos + xlen + 1 == slen || s[pos + xlen + 1] != '$') {
      li_assign(c, 'n', s + pos, 1);
      return pos + 1;
    }
    // my_memmem(cs + xlen + 2, slen - (pos + xlen + 2), cs + pos, xlen + 2): the
    // haystack starts at xlen + 2, as in the C source
    const uint32_t nl = xlen + 2, hb = xlen + 2, he = xlen + 2 + (slen - (pos + xlen + 2));
    int64_t e = -1;
    for (uint32_t h = hb; h + nl <= he && e < 0; h++) {
      bool m = true;
      for (uint32_t k = 0; k < nl && m; k++) m = s[h + k] == s[pos + k];
      if (m) e = h;
    }
    c.sopen = '$';
    if (e < 0 || (uint32_t)e < pos + xlen + 2) {
      li_assign(c, 's', s + pos + xlen + 2, slen - pos - xlen - 2);
      c.sclose = 0;
      return slen;
    }
    li_assign(c, 's', s + pos + xlen + 2, (uint32_t)e - (pos + xlen + 2));
    c.sclose = '$';
    return (uint32_t)e + xlen + 2;
  }
  if (xlen == 1 && s[pos + 1] == '.') return li_parse_word(S, c, pos);
  li_assign(c, '1', s + pos, 1 + xlen);
  return pos + 1 + xlen;
}

GI_HD __forceinline__ uint32_t li_parse_number(LiSqli& S, LiTok& c, uint32_t pos) {
  const uint8_t* s = S.s;
  const uint32_t slen = S.slen;
  if (s[pos] == '0' && pos + 1 < slen) {
    int kind = 0;  // 1 hex, 2 binary
    if (s[pos + 1] == 'X' || s[pos + 1] == 'x') kind = 1;
    else if (s[pos + 1] == 'B' || s[pos + 1] == 'b') kind = 2;
    if (kind) {
      uint32_t xlen = 0;
      while (pos + 2 + xlen < slen &&
             (kind == 1 ? li_ishex(s[pos + 2 + xlen]) : (s[pos + 2 + xlen] == '0' || s[pos + 2 + xlen] == '1')))
        xlen++;
      if (xlen == 0) {
        li_assign(c, 'n', s + pos, 2);
        return pos + 2;
      }
      li_assign(c, '1', s + pos, 2 + xlen);
      return pos + 2 + xlen;
    }
  }
  const uint32_t start = pos;
  while (pos < slen && li_isdigit(s[pos])) pos++;
  if (pos < slen && s[pos] == '.') {
    pos++;
    while (pos < slen && li_isdigit(s[pos])) pos++;
    if (pos - start == 1) {
      li_assign(c, '.', s + start, 1);
      return pos;
    }
  }
  bool have_e = false, have_exp = false;
  if (pos < slen && (s[pos] == 'E' || s[pos] == 'e')) {
    have_e = true;
    pos++;
    if (pos < slen && (s[pos] == '+' || s[pos] == '-')) pos++;
    while (pos < slen && li_isdigit(s[pos])) {
      have_exp = true;
      pos++;
    }
  }
  if (pos < slen && (s[pos] == 'd' || s[pos] == 'D' || s[pos] == 'f' || s[pos] == 'F')) {
    if (pos + 1 == slen) pos++;
    else if (li_white(s[pos + 1]) || s[pos + 1] == ';') pos++;
    else if (s[pos + 1] == 'u' || s[pos + 1] == 'U') pos++;
  }
  li_assign(c, (have_e && !have_exp) ? 'n' : '1', s + start, pos - start);
  return pos;
}

// one parser step at S.pos into token c: returns the new position
GI_HD __forceinline__ uint32_t li_parse(LiSqli& S, LiTok& c) {
  const uint8_t* s = S.s;
  const uint32_t slen = S.slen, pos = S.pos;
  const uint8_t ch = s[pos];
  switch (li_parser(ch)) {
    case LP_WHITE: return pos + 1;
    case LP_OP1: li_assign(c, 'o', s + pos, 1); return pos + 1;
    case LP_OTHER: li_assign(c, '?', s + pos, 1); return pos + 1;
    case LP_CHAR: li_assign(c, ch, s + pos, 1); return pos + 1;
    case LP_STRING: return li_string_core(s, slen, pos, c, ch, 1);
    case LP_HASH:
      S.hash++;
      if (S.flags & LI_FLAG_SQL_MYSQL) {
        S.hash++;
        return li_parse_eol_comment(S, c, pos);
      }
      li_assign(c, 'o', s + pos, 1);
      return pos + 1;
    case LP_DASH:
      if (pos + 2 < slen && s[pos + 1] == '-' && li_white(s[pos + 2])) return li_parse_eol_comment(S, c, pos);
      if (pos + 2 == slen && s[pos + 1] == '-') return li_parse_eol_comment(S, c, pos);
      if (pos + 1 < slen && s[pos + 1] == '-' && (S.flags & LI_FLAG_SQL_ANSI)) {
        S.ddx++;
        return li_parse_eol_comment(S, c, pos);
      }
      li_assign(c, 'o', s + pos, 1);
      return pos + 1;
    case LP_SLASH: {
      if (pos + 1 == slen || s[pos + 1] != '*') {
        li_assign(c, 'o', s + pos, 1);
        return pos + 1;
      }
      const int64_t ptr = li_memchr2(s, pos + 2, slen, '*', '/');
      const uint32_t clen = ptr < 0 ? slen - pos : (uint32_t)ptr + 2 - pos;
      const uint32_t inner_end = ptr < 0 ? slen : (uint32_t)ptr + 1;
      uint8_t ty = 'c';
      if (li_memchr2(s, pos + 2, inner_end, '/', '*') >= 0) ty = 'X';
      else if (pos + 2 < slen && s[pos + 2] == '!') ty = 'X';
      li_assign(c, ty, s + pos, clen);
      return pos + clen;
    }
    case LP_BACKSLASH:
      if (pos + 1 < slen && s[pos + 1] == 'N') {
        li_assign(c, '1', s + pos, 2);
        return pos + 2;
      }
      li_assign(c, '\\', s + pos, 1);
      return pos + 1;
    case LP_OP2: {
      if (pos + 1 >= slen) {
        li_assign(c, 'o', s + pos, 1);
        return pos + 1;
      }
      if (pos + 2 < slen && s[pos] == '<' && s[pos + 1] == '=' && s[pos + 2] == '>') {
        li_assign(c, 'o', s + pos, 3);
        return pos + 3;
      }
      const uint8_t t = li_lookup(LI_T(S), s + pos, 2);
      if (t) {
        li_assign(c, t, s + pos, 2);
        return pos + 2;
      }
      li_assign(c, s[pos] == ':' ? ':' : 'o', s + pos, 1);
      return pos + 1;
    }
    case LP_NUMBER: return li_parse_number(S, c, pos);
    case LP_MONEY: return li_parse_money(S, c, pos);
    case LP_VAR: {
      uint32_t p = pos + 1;
      if (p < slen && s[p] == '@') p++;
      if (p < slen) {
        if (s[p] == '`') {
          const uint32_t np = li_parse_tick(S, c, p);
          c.type = 'v';
          return np;
        }
        if (s[p] == '\'' || s[p] == '"') {
          const uint32_t np = li_string_core(s, slen, p, c, s[p], 1);
          c.type = 'v';
          return np;
        }
      }
      uint32_t e = p;
      while (e < slen && !li_var_stop(s[e])) e++;
      li_assign(c, 'v', s + p, e - p);
      return e;
    }
    case LP_BSTRING:
    case LP_XSTRING: {
      if (pos + 2 >= slen || s[pos + 1] != '\'') return li_parse_word(S, c, pos);
      const bool hex = li_parser(ch) == LP_XSTRING;
      uint32_t wlen = 0;
      while (pos + 2 + wlen < slen && (hex ? li_ishex(s[pos + 2 + wlen]) : (s[pos + 2 + wlen] == '0' || s[pos + 2 + wlen] == '1')))
        wlen++;
      if (pos + 2 + wlen >= slen || s[pos + 2 + wlen] != '\'') return li_parse_word(S, c, pos);
      li_assign(c, '1', s + pos, wlen + 3);
      return pos + 2 + wlen + 1;
    }
    case LP_ESTRING: return li_parse_estring(S, c, pos);
    case LP_NQSTRING:
      if (pos + 2 < slen && s[pos + 1] == '\'') return li_parse_estring(S, c, pos);
      return li_parse_qstring_core(S, c, pos, 1);
    case LP_QSTRING: return li_parse_qstring_core(S, c, pos, 0);
    case LP_USTRING:
      if (pos + 2 < slen && s[pos + 1] == '&' && s[pos + 2] == '\'') {
        const uint32_t np = li_string_core(s, slen, pos + 2, c, '\'', 1);
        c.sopen = 'u';
        if (c.sclose == '\'') c.sclose = 'u';
        return np;
      }
      return li_parse_word(S, c, pos);
    case LP_BWORD: {
      const int64_t e = li_memchr(s, pos, slen, ']');
      if (e < 0) {
        li_assign(c, 'n', s + pos, slen - pos);
        return slen;
      }
      li_assign(c, 'n', s + pos, (uint32_t)e - pos + 1);
      return (uint32_t)e + 1;
    }
    case LP_TICK: return li_parse_tick(S, c, pos);
    default: return li_parse_word(S, c, pos);
  }
}

// libinjection_sqli_tokenize into tv[S.cur]
GI_HD __forceinline__ bool li_tokenize(LiSqli& S) {
  if (S.slen == 0) return false;
  LiTok& c = S.tv[S.cur];
  li_clear(c);
  if (S.pos == 0 && (S.flags & (LI_FLAG_QUOTE_SINGLE | LI_FLAG_QUOTE_DOUBLE))) {
    S.pos = li_string_core(S.s, S.slen, 0, c, (S.flags & LI_FLAG_QUOTE_SINGLE) ? '\'' : '"', 0);
    S.ntok++;
    return true;
  }
  while (S.pos < S.slen) {
    S.pos = li_parse(S, c);
    if (c.type) {
      S.ntok++;
      return true;
    }
  }
  return false;
}

GI_HD __forceinline__ bool li_unary(const LiTok& t) {  // st_is_unary_op
  if (t.type != 'o') return false;
  if (t.len == 1) return t.p[0] == '+' || t.p[0] == '-' || t.p[0] == '!' || t.p[0] == '~';
  if (t.len == 2) return t.p[0] == '!' && t.p[1] == '!';
  if (t.len == 3) return li_tok_is(t, "NOT");
  return false;
}
GI_HD __forceinline__ bool li_arith(const LiTok& t) {
  const uint8_t ch = t.len ? t.p[0] : 0;
  return t.type == 'o' && t.len == 1 && (ch == '*' || ch == '/' || ch == '-' || ch == '+' || ch == '%');
}
GI_HD __forceinline__ bool li_in(uint8_t c, const char* set) {
  for (uint32_t i = 0; set[i]; i++)
    if ((uint8_t)set[i] == c) return true;
  return false;
}

// syntax_merge_words: a's value becomes the keyword pool entry of "a b"
GI_HD __forceinline__ bool li_merge(const LiTables& T, LiTok& a, const LiTok& b) {
  if (!li_in(a.type, "knoUfETt") || !li_in(b.type, "knoUfETt&")) return false;
  const uint32_t sz3 = (uint32_t)a.len + b.len + 1;
  if (sz3 >= LI_TOKEN_SIZE) return false;
  const int i = li_find(T, a.p, a.len, b.p, b.len, true);
  if (i < 0) return false;
  const uint32_t e = T.words[i];
  a.type = (uint8_t)(e >> 24);
  a.p = T.pool + (e & 0xFFFFu);  // the pool copy of the merged word (same bytes up to case)
  a.len = (uint16_t)sz3;
  return true;
}

GI_HD __forceinline__ bool li_func_word(const LiTok& t) {
  return li_tok_is(t, "USER_ID") || li_tok_is(t, "USER_NAME") || li_tok_is(t, "DATABASE") ||
         li_tok_is(t, "PASSWORD") || li_tok_is(t, "USER") || li_tok_is(t, "CURRENT_USER") ||
         li_tok_is(t, "CURRENT_DATE") || li_tok_is(t, "CURRENT_TIME") || li_tok_is(t, "CURRENT_TIMESTAMP") ||
         li_tok_is(t, "LOCALTIME") || li_tok_is(t, "LOCALTIMESTAMP");
}

// the next token into tv[pos] (comments go to last_comment): libinjection_sqli_fold's inner loops
GI_HD __forceinline__ void li_pull(LiSqli& S, uint32_t& pos, bool& more, LiTok& last) {
  S.cur = pos;
  more = li_tokenize(S);
  if (more) {
    if (S.tv[pos].type == 'c') {
      last = S.tv[pos];
    } else {
      last.type = 0;
      pos++;
    }
  }
}

// libinjection_sqli_fold -> number of fingerprint tokens
GI_HD __noinline__ uint32_t li_fold(LiSqli& S) {
  LiTok* tv = S.tv;
  uint32_t pos = 0, left = 0;
  bool more = true;
  LiTok last;
  li_clear(last);
  S.cur = 0;
  while (more) {
    more = li_tokenize(S);
    const LiTok& c = tv[0];
    if (!(c.type == 'c' || c.type == '(' || c.type == 't' || li_unary(c))) break;
  }
  if (!more) return 0;
  pos = 1;
  for (uint32_t guard = 0; guard < 8 * S.slen + 64; guard++) {  // never reached: every pass consumes or folds
    if (pos >= LI_MAX_TOKENS) {
      const uint8_t t0 = tv[0].type, t1 = tv[1].type, t2 = tv[2].type, t3 = tv[3].type, t4 = tv[4].type;
      if ((t0 == '1' && (t1 == 'o' || t1 == ',') && t2 == '(' && t3 == '1' && t4 == ')') ||
          (t0 == 'n' && t1 == 'o' && t2 == '(' && (t3 == 'n' || t3 == '1') && t4 == ')') ||
          (t0 == '1' && t1 == ')' && t2 == ',' && t3 == '(' && t4 == '1') ||
          (t0 == 'n' && t1 == ')' && t2 == 'o' && t3 == '(' && t4 == 'n')) {
        if (pos > LI_MAX_TOKENS) {
          tv[1] = tv[LI_MAX_TOKENS];
          pos = 2;
        } else {
          pos = 1;
        }
        left = 0;
      }
    }
    if (!more || left >= LI_MAX_TOKENS) {
      left = pos;
      break;
    }
    while (more && pos <= LI_MAX_TOKENS && pos - left < 2) li_pull(S, pos, more, last);
    if (pos - left < 2) {
      left = pos;
      continue;
    }
    LiTok& a = tv[left];
    LiTok& b = tv[left + 1];
    if (a.type == 's' && b.type == 's') { pos--; continue; }
    if (a.type == ';' && b.type == ';') { pos--; continue; }
    if ((a.type == 'o' || a.type == '&') && (li_unary(b) || b.type == 't')) { pos--; left = 0; continue; }
    if (a.type == '(' && li_unary(b)) { pos--; if (left > 0) left--; continue; }
    if (li_merge(LI_T(S), a, b)) { pos--; if (left > 0) left--; continue; }
    if (a.type == ';' && b.type == 'f' && b.len >= 2 && (b.p[0] == 'I' || b.p[0] == 'i') && (b.p[1] == 'F' || b.p[1] == 'f')) {
      b.type = 'T';
      continue;
    }
    if ((a.type == 'n' || a.type == 'v') && b.type == '(' && li_func_word(a)) { a.type = 'f'; continue; }
    if (a.type == 'k' && (li_tok_is(a, "IN") || li_tok_is(a, "NOT IN"))) {
      a.type = b.type == '(' ? 'o' : 'n';
      continue;
    }
    bool fall3 = true;
    if (a.type == 'o' && (li_tok_is(a, "LIKE") || li_tok_is(a, "NOT LIKE"))) {
      if (b.type == '(') a.type = 'f';
    } else if (a.type == 't' && li_in(b.type, "n1t(fvs")) {
      a = b;
      pos--;
      left = 0;
      continue;
    } else if (a.type == 'A' && b.type == 'n') {
      bool us = false;
      for (uint32_t i = 0; i < b.len; i++) us |= b.p[i] == '_';
      if (us) {
        b.type = 't';
        left = 0;
      }
    } else if (a.type == '\\') {
      if (li_arith(b)) {
        a.type = '1';
      } else {
        a = b;
        pos--;
      }
      left = 0;
      continue;
    } else if (a.type == '(' && b.type == '(') {
      pos--; left = 0; continue;
    } else if (a.type == ')' && b.type == ')') {
      pos--; left = 0; continue;
    } else if (a.type == '{' && b.type == 'n') {
      if (b.len == 0) {
        b.type = 'X';
        return left + 2;
      }
      left = 0;
      pos -= 2;
      continue;
    } else if (b.type == '}') {
      pos--; left = 0; continue;
    }
    (void)fall3;
    while (more && pos <= LI_MAX_TOKENS && pos - left < 3) li_pull(S, pos, more, last);
    if (pos - left < 3) {
      left = pos;
      continue;
    }
    LiTok& x = tv[left];
    LiTok& y = tv[left + 1];
    LiTok& z = tv[left + 2];
    if (x.type == '1' && y.type == 'o' && z.type == '1') { pos -= 2; left = 0; continue; }
    if (x.type == 'o' && y.type != '(' && z.type == 'o') { left = 0; pos -= 2; continue; }
    if (x.type == '&' && z.type == '&') { pos -= 2; left = 0; continue; }
    if (x.type == 'v' && y.type == 'o' && li_in(z.type, "v1n")) { pos -= 2; left = 0; continue; }
    if ((x.type == 'n' || x.type == '1') && y.type == 'o' && (z.type == '1' || z.type == 'n')) { pos -= 2; left = 0; continue; }
    if (li_in(x.type, "n1vs") && y.type == 'o' && y.len == 2 && y.p[0] == ':' && y.p[1] == ':' && z.type == 't') {
      pos -= 2; left = 0; continue;
    }
    if (li_in(x.type, "n1sv") && y.type == ',' && li_in(z.type, "1nsv")) { pos -= 2; left = 0; continue; }
    if (li_in(x.type, "EB,") && li_unary(y) && z.type == '(') { y = z; pos--; left = 0; continue; }
    if (li_in(x.type, "kEB") && li_unary(y) && li_in(z.type, "1nvsf")) { y = z; pos--; left = 0; continue; }
    if (x.type == ',' && li_unary(y) && li_in(z.type, "1nvs")) { y = z; left = 0; pos -= 3; continue; }
    if (x.type == ',' && li_unary(y) && z.type == 'f') { y = z; pos--; left = 0; continue; }
    if (x.type == 'n' && y.type == '.' && z.type == 'n') { pos -= 2; left = 0; continue; }
    if (x.type == 'E' && y.type == '.' && z.type == 'n') { y = z; pos--; left = 0; continue; }
    if (x.type == 'f' && y.type == '(' && z.type != ')') {
      if (li_tok_is(x, "USER")) x.type = 'n';
    }
    left++;
  }
  if (left < LI_MAX_TOKENS && last.type == 'c') {
    tv[left] = last;
    left++;
  }
  if (left > LI_MAX_TOKENS) left = LI_MAX_TOKENS;
  return left;
}

// fingerprint blacklist: the authored grammar of libinj_tables.FINGERPRINT_RULES
// (f upper-cased, n <= 5), matched by hand
GI_HD __noinline__ bool li_fp_black(const uint8_t* f, uint32_t n) {
  if (n == 0) return false;
  auto at = [&](uint32_t i) -> uint8_t { return i < n ? f[i] : (uint8_t)0; };
  auto val1s = [&](uint8_t c) { return c == '1' || c == 'S'; };
  auto val1sn = [&](uint8_t c) { return c == '1' || c == 'S' || c == 'N'; };
  auto vsvf = [&](uint8_t c) { return c == '1' || c == 'S' || c == 'V' || c == 'F'; };
  const uint8_t f0 = f[0];
  if (n == 1 && f0 == 'X') return true;                                           // R1
  for (uint32_t i = 0; i < n; i++) {
    if (f[i] == 'U' && (at(i + 1) == 'E' || (at(i + 1) == '(' && at(i + 2) == 'E'))) return true;  // R2
    if (f[i] == ';' && (at(i + 1) == 'E' || at(i + 1) == 'T')) return true;                         // R3
  }
  uint32_t i = 1;
  while (at(i) == ')') i++;
  const uint32_t nclose = i - 1;
  const uint8_t op = at(i);
  uint32_t j = i + 1;
  while (at(j) == '(') j++;
  if (val1s(f0) && (op == '&' || op == 'O') && vsvf(at(j))) return true;          // R4
  if (f0 == 'N' && op == '&' && vsvf(at(j))) return true;                         // R5
  if (n == 2 && val1sn(f0) && f[1] == 'C') return true;                           // R6
  if (f0 == 'E') {                                                                // R7
    uint32_t k = 1;
    while (at(k) == '(') k++;
    if (vsvf(at(k))) return true;
    if (at(1) == 'K' || at(2) == 'K' || at(3) == 'K') return true;
    if ((at(1) == '1' || at(1) == 'S' || at(1) == 'N' || at(1) == 'V') && at(2) == ',') return true;
  }
  if (val1sn(f0)) {
    if (op == 'B' && li_in(at(i + 1), "1NS(") && at(i + 1) != 0) return true;     // R8
    if (nclose >= 1 && (op == '&' || op == 'O' || op == ';' || op == 'U')) return true;  // R9
    if (op == 'U') return true;                                                    // R12
    if (f[1] == 'K' && (at(2) == 'S' || at(2) == '1')) return true;               // R13
  }
  if (f0 == '&') {                                                                // R10
    uint32_t k = 1;
    while (at(k) == '(') k++;
    if (vsvf(at(k))) return true;
  }
  if (f0 == 'T' && li_in(at(1), "N1SVF(") && at(1) != 0) return true;            // R11
  if (f0 == 'F' && at(1) == '(') {                                                 // R14
    if (at(2) == ')') return true;
    if (li_in(at(2), "1SNV") && at(2) != 0 && at(3) == ')') return true;
  }
  return false;
}

GI_HD __forceinline__ uint8_t li_fpc(const LiSqli& S, uint32_t i) { return S.tv[i].type; }

// libinjection_sqli_not_whitelist (fp = the fingerprint, tlen tokens)
GI_HD __noinline__ bool li_not_whitelist(const LiSqli& S, const uint8_t* fp, uint32_t tlen) {
  const LiTok* tv = S.tv;
  if (tlen > 1 && fp[tlen - 1] == 'c') {
    const uint8_t* s = S.s;
    for (uint32_t i = 0; i + 11 <= S.slen; i++) {
      bool m = true;
      const char* w = "sp_password";
      for (uint32_t k = 0; k < 11 && m; k++) m = s[i + k] == (uint8_t)w[k];
      if (m) return true;
    }
  }
  auto sat = [&](uint32_t i) -> uint8_t { return i < S.slen ? S.s[i] : (uint8_t)0; };
  if (tlen == 2) {
    if (fp[1] == 'U') return S.ntok != 2;
    if (tv[1].len && tv[1].p[0] == '#') return false;
    if (tv[0].type == 'n' && tv[1].type == 'c' && !(tv[1].len && tv[1].p[0] == '/')) return false;
    if (tv[0].type == '1' && tv[1].type == 'c' && tv[1].len && tv[1].p[0] == '/') return true;
    if (tv[0].type == '1' && tv[1].type == 'c') {
      if (S.ntok > 2) return true;
      const uint8_t ch = sat(tv[0].len);
      if (ch <= 32) return true;
      if (ch == '/' && sat(tv[0].len + 1) == '*') return true;
      if (ch == '-' && sat(tv[0].len + 1) == '-') return true;
      return false;
    }
    if (tv[1].len > 2 && tv[1].p[0] == '-') return false;
  } else if (tlen == 3) {
    const bool sos = fp[0] == 's' && fp[2] == 's' && (fp[1] == 'o' || fp[1] == '&');
    if (sos) {
      return tv[0].sopen == 0 && tv[2].sclose == 0 && tv[0].sclose == tv[2].sopen;
    }
    const bool pair = (fp[0] == 's' && fp[1] == '&' && fp[2] == 'n') || (fp[0] == 'n' && fp[1] == '&' && fp[2] == '1') ||
                      (fp[0] == '1' && fp[1] == '&' && (fp[2] == '1' || fp[2] == 'v' || fp[2] == 's'));
    if (pair) {
      if (S.ntok == 3) return false;
    } else if (tv[1].type == 'k') {
      bool into = tv[1].len >= 4;
      for (uint32_t k = 0; k < 4 && into; k++) into = li_up(tv[1].p[k]) == (uint8_t)"INTO"[k];
      if (tv[1].len < 5 || !into) return false;
    }
  }
  return true;
}

// libinjection_sqli_fingerprint + the blacklist/whitelist check for one context
GI_HD __noinline__ bool li_sqli_ctx(LiSqli& S, uint32_t flags) {
  S.flags = flags;
  S.pos = 0;
  S.cur = 0;
  S.ddx = S.hash = S.ntok = 0;
  for (uint32_t k = 0; k < 8; k++) li_clear(S.tv[k]);
  uint32_t tlen = li_fold(S);
  if (tlen > 2 && S.tv[tlen - 1].type == 'n' && S.tv[tlen - 1].sopen == '`' && S.tv[tlen - 1].len == 0 &&
      S.tv[tlen - 1].sclose == 0)
    S.tv[tlen - 1].type = 'c';
  uint8_t fp[8];
  bool evil = false;
  for (uint32_t i = 0; i < tlen; i++) {
    fp[i] = S.tv[i].type;
    evil |= fp[i] == 'X';
  }
  if (evil) {
    tlen = 1;
    fp[0] = 'X';
    S.tv[0].type = 'X';
    S.tv[0].p = (const uint8_t*)"X";
    S.tv[0].len = 1;
    S.tv[1].type = 0;
  }
  uint8_t up[8];
  for (uint32_t i = 0; i < tlen; i++) up[i] = li_up(fp[i]);
  return li_fp_black(up, tlen) && li_not_whitelist(S, fp, tlen);
}

// libinjection_is_sqli.  `st` is the caller's state buffer (LDS in k_detect,
// the request's macro scratch in k_eval): kept in memory, the tokenizer state
// does not inflate the register budget of every kernel that can call this.
GI_HD __noinline__ bool li_detect_sqli(const uint8_t* s, uint32_t n, LiSqli* st, const LiTables& T) {
  if (n == 0) return false;
  LiSqli& S = *st;
#ifndef LI_LDS_TABLES
  S.T = T;
#else
  (void)T;
#endif
  S.s = s;
  S.slen = n;
  if (li_sqli_ctx(S, LI_FLAG_QUOTE_NONE | LI_FLAG_SQL_ANSI)) return true;
  if ((S.ddx || S.hash) && li_sqli_ctx(S, LI_FLAG_QUOTE_NONE | LI_FLAG_SQL_MYSQL)) return true;
  bool sq = false, dq = false;
  for (uint32_t i = 0; i < n; i++) {
    sq |= s[i] == '\'';
    dq |= s[i] == '"';
  }
  if (sq) {
    if (li_sqli_ctx(S, LI_FLAG_QUOTE_SINGLE | LI_FLAG_SQL_ANSI)) return true;
    if ((S.ddx || S.hash) && li_sqli_ctx(S, LI_FLAG_QUOTE_SINGLE | LI_FLAG_SQL_MYSQL)) return true;
  }
  if (dq && li_sqli_ctx(S, LI_FLAG_QUOTE_DOUBLE | LI_FLAG_SQL_MYSQL)) return true;
  return false;
}

// Exact prefilter: a value whose bytes are all in [A-Za-z0-9_] tokenizes to at
// most two tokens (a number, then one word running to the end: the word stop
// set has none of these bytes, and the quote contexts need a quote), and no
// two-token fingerprint of that shape survives blacklist + whitelist (the only
// blacklisted one, value + UNION, is whitelisted at two tokens) -- so it is
// never SQLi.  tests/test_libinjection.py checks the claim on a corpus.
GI_HD __forceinline__ bool li_sqli_byte(uint8_t c) {
  return !((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_');
}
// Exact prefilter: without any of  NUL \t \n \v \f \r space < > = ' " ` /
// each of the five start states yields a single DATA_TEXT / ATTR_NAME /
// ATTR_VALUE token with no black attribute before it -- never XSS.
GI_HD __forceinline__ bool li_xss_byte(uint8_t c) {
  return c == 0 || (c >= 9 && c <= 13) || c == ' ' || c == '<' || c == '>' || c == '=' || c == '\'' || c == '"' ||
         c == '`' || c == '/';
}
GI_HD inline bool li_candidate(bool sqli, const uint8_t* s, uint32_t n) {
  for (uint32_t i = 0; i < n; i++)
    if (sqli ? li_sqli_byte(s[i]) : li_xss_byte(s[i])) return true;
  return false;
}

// -------------------------------------------------------------- XSS ----
enum : uint8_t {
  H5_DATA_TEXT, H5_TAG_NAME_OPEN, H5_TAG_NAME_CLOSE, H5_TAG_NAME_SELFCLOSE, H5_TAG_DATA, H5_TAG_CLOSE,
  H5_ATTR_NAME, H5_ATTR_VALUE, H5_TAG_COMMENT, H5_DOCTYPE,
};
enum : uint8_t {  // h5 states
  HS_EOF, HS_DATA, HS_TAG_OPEN, HS_END_TAG_OPEN, HS_TAG_NAME_CLOSE, HS_TAG_NAME, HS_BEFORE_ATTR_NAME,
  HS_ATTR_NAME, HS_AFTER_ATTR_NAME, HS_BEFORE_ATTR_VALUE, HS_VALUE_DQ, HS_VALUE_SQ, HS_VALUE_BQ,
  HS_VALUE_NQ, HS_AFTER_VALUE_QUOTED, HS_SELF_CLOSING, HS_BOGUS_COMMENT, HS_BOGUS_COMMENT2,
  HS_MARKUP_DECL_OPEN, HS_COMMENT, HS_CDATA, HS_DOCTYPE,
};

struct H5 {
  const uint8_t* s;
  uint32_t len, pos;
  uint32_t ts, tl;  // token start, length
  uint8_t tt, state, is_close, _pad;
};

GI_HD __forceinline__ bool h5_white(uint8_t c) {  // strchr(" \t\n\v\f\r", ch): NUL matches the terminator
  return c == ' ' || (c >= 9 && c <= 13) || c == 0;
}
GI_HD __forceinline__ bool h5_alpha(uint8_t c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
GI_HD __forceinline__ void h5_tok(H5& h, uint32_t st, uint32_t n, uint8_t t) {
  h.ts = st;
  h.tl = n;
  h.tt = t;
}
// h5_skip_white: next non-white byte, -1 at the end
GI_HD __forceinline__ int h5_skip_white(H5& h) {
  while (h.pos < h.len) {
    const uint8_t c = h.s[h.pos];
    if (c == 0 || c == ' ' || (c >= 9 && c <= 13)) h.pos++;
    else return c;
  }
  return -1;
}

// libinjection_h5_next: one token (false at the end).  `run` is the state
// code to execute (a C tail call jumps to another state's code without
// changing the persistent h.state).
GI_HD __noinline__ bool h5_next(H5& h) {
  uint8_t run = h.state;
  const uint8_t* s = h.s;
  for (uint32_t guard = 0; guard < 64; guard++) {
    switch (run) {
      case HS_EOF: return false;
      case HS_DATA: {
        const int64_t i = li_memchr(s, h.pos, h.len, '<');
        if (i < 0) {
          h5_tok(h, h.pos, h.len - h.pos, H5_DATA_TEXT);
          h.state = HS_EOF;
          if (h.tl == 0) return false;
        } else {
          h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_DATA_TEXT);
          h.pos = (uint32_t)i + 1;
          h.state = HS_TAG_OPEN;
          if (h.tl == 0) { run = HS_TAG_OPEN; continue; }
        }
        return true;
      }
      case HS_TAG_OPEN: {
        if (h.pos >= h.len) return false;
        const uint8_t ch = s[h.pos];
        if (ch == '!') { h.pos++; run = HS_MARKUP_DECL_OPEN; continue; }
        if (ch == '/') { h.pos++; h.is_close = 1; run = HS_END_TAG_OPEN; continue; }
        if (ch == '?') { h.pos++; run = HS_BOGUS_COMMENT; continue; }
        if (ch == '%') { h.pos++; run = HS_BOGUS_COMMENT2; continue; }
        if (h5_alpha(ch) || ch == 0) { run = HS_TAG_NAME; continue; }
        if (h.pos == 0) { run = HS_DATA; continue; }
        h5_tok(h, h.pos - 1, 1, H5_DATA_TEXT);
        h.state = HS_DATA;
        return true;
      }
      case HS_END_TAG_OPEN: {
        if (h.pos >= h.len) return false;
        const uint8_t ch = s[h.pos];
        if (ch == '>') { run = HS_DATA; continue; }
        if (h5_alpha(ch)) { run = HS_TAG_NAME; continue; }
        h.is_close = 0;
        run = HS_BOGUS_COMMENT;
        continue;
      }
      case HS_TAG_NAME_CLOSE:
        h.is_close = 0;
        h5_tok(h, h.pos, 1, H5_TAG_NAME_CLOSE);
        h.pos++;
        h.state = h.pos < h.len ? HS_DATA : HS_EOF;
        return true;
      case HS_TAG_NAME: {
        uint32_t p = h.pos;
        while (p < h.len) {
          const uint8_t ch = s[p];
          if (ch == 0) {
            p++;
          } else if (h5_white(ch)) {
            h5_tok(h, h.pos, p - h.pos, H5_TAG_NAME_OPEN);
            h.pos = p + 1;
            h.state = HS_BEFORE_ATTR_NAME;
            return true;
          } else if (ch == '/') {
            h5_tok(h, h.pos, p - h.pos, H5_TAG_NAME_OPEN);
            h.pos = p + 1;
            h.state = HS_SELF_CLOSING;
            return true;
          } else if (ch == '>') {
            h5_tok(h, h.pos, p - h.pos, H5_TAG_NAME_OPEN);
            if (h.is_close) {
              h.pos = p + 1;
              h.is_close = 0;
              h.tt = H5_TAG_CLOSE;
              h.state = HS_DATA;
            } else {
              h.pos = p;
              h.state = HS_TAG_NAME_CLOSE;
            }
            return true;
          } else {
            p++;
          }
        }
        h5_tok(h, h.pos, h.len - h.pos, H5_TAG_NAME_OPEN);
        h.state = HS_EOF;
        return true;
      }
      case HS_BEFORE_ATTR_NAME: {
        const int ch = h5_skip_white(h);
        if (ch == -1) return false;
        if (ch == '/') { h.pos++; run = HS_SELF_CLOSING; continue; }
        if (ch == '>') {
          h.state = HS_DATA;
          h5_tok(h, h.pos, 1, H5_TAG_NAME_CLOSE);
          h.pos++;
          return true;
        }
        run = HS_ATTR_NAME;
        continue;
      }
      case HS_ATTR_NAME: {
        uint32_t p = h.pos + 1;
        while (p < h.len) {
          const uint8_t ch = s[p];
          if (h5_white(ch) || ch == '/' || ch == '=' || ch == '>') {
            h5_tok(h, h.pos, p - h.pos, H5_ATTR_NAME);
            if (ch == '>') {
              h.state = HS_TAG_NAME_CLOSE;
              h.pos = p;
            } else {
              h.state = ch == '/' ? HS_SELF_CLOSING : ch == '=' ? HS_BEFORE_ATTR_VALUE : HS_AFTER_ATTR_NAME;
              h.pos = p + 1;
            }
            return true;
          }
          p++;
        }
        h5_tok(h, h.pos, h.len - h.pos, H5_ATTR_NAME);
        h.state = HS_EOF;
        h.pos = h.len;
        return true;
      }
      case HS_AFTER_ATTR_NAME: {
        const int ch = h5_skip_white(h);
        if (ch == -1) return false;
        if (ch == '/') { h.pos++; run = HS_SELF_CLOSING; continue; }
        if (ch == '=') { h.pos++; run = HS_BEFORE_ATTR_VALUE; continue; }
        if (ch == '>') { run = HS_TAG_NAME_CLOSE; continue; }
        run = HS_ATTR_NAME;
        continue;
      }
      case HS_BEFORE_ATTR_VALUE: {
        const int ch = h5_skip_white(h);
        if (ch == -1) {
          h.state = HS_EOF;
          return false;
        }
        run = ch == '"' ? HS_VALUE_DQ : ch == '\'' ? HS_VALUE_SQ : ch == '`' ? HS_VALUE_BQ : HS_VALUE_NQ;
        continue;
      }
      case HS_VALUE_DQ:
      case HS_VALUE_SQ:
      case HS_VALUE_BQ: {
        const uint8_t q = run == HS_VALUE_DQ ? '"' : run == HS_VALUE_SQ ? '\'' : '`';
        if (h.pos > 0) h.pos++;
        const int64_t i = li_memchr(s, h.pos, h.len, q);
        if (i < 0) {
          h5_tok(h, h.pos, h.len - h.pos, H5_ATTR_VALUE);
          h.state = HS_EOF;
        } else {
          h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_ATTR_VALUE);
          h.state = HS_AFTER_VALUE_QUOTED;
          h.pos += h.tl + 1;
        }
        return true;
      }
      case HS_VALUE_NQ: {
        uint32_t p = h.pos;
        while (p < h.len) {
          const uint8_t ch = s[p];
          if (h5_white(ch)) {
            h5_tok(h, h.pos, p - h.pos, H5_ATTR_VALUE);
            h.pos = p + 1;
            h.state = HS_BEFORE_ATTR_NAME;
            return true;
          }
          if (ch == '>') {
            h5_tok(h, h.pos, p - h.pos, H5_ATTR_VALUE);
            h.pos = p;
            h.state = HS_TAG_NAME_CLOSE;
            return true;
          }
          p++;
        }
        h.state = HS_EOF;
        h5_tok(h, h.pos, h.len - h.pos, H5_ATTR_VALUE);
        return true;
      }
      case HS_AFTER_VALUE_QUOTED: {
        if (h.pos >= h.len) return false;
        const uint8_t ch = s[h.pos];
        if (h5_white(ch)) { h.pos++; run = HS_BEFORE_ATTR_NAME; continue; }
        if (ch == '/') { h.pos++; run = HS_SELF_CLOSING; continue; }
        if (ch == '>') {
          h5_tok(h, h.pos, 1, H5_TAG_NAME_CLOSE);
          h.pos++;
          h.state = HS_DATA;
          return true;
        }
        run = HS_BEFORE_ATTR_NAME;
        continue;
      }
      case HS_SELF_CLOSING: {
        if (h.pos >= h.len) return false;
        if (s[h.pos] == '>') {
          h5_tok(h, h.pos - 1, 2, H5_TAG_NAME_SELFCLOSE);
          h.state = HS_DATA;
          h.pos++;
          return true;
        }
        run = HS_BEFORE_ATTR_NAME;
        continue;
      }
      case HS_BOGUS_COMMENT: {
        const int64_t i = li_memchr(s, h.pos, h.len, '>');
        if (i < 0) {
          h5_tok(h, h.pos, h.len - h.pos, H5_TAG_COMMENT);
          h.pos = h.len;
          h.state = HS_EOF;
        } else {
          h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_TAG_COMMENT);
          h.pos = (uint32_t)i + 1;
          h.state = HS_DATA;
        }
        return true;
      }
      case HS_BOGUS_COMMENT2: {
        uint32_t p = h.pos;
        while (true) {
          const int64_t i = li_memchr(s, p, h.len, '%');
          if (i < 0 || (uint32_t)i + 1 >= h.len) {
            h5_tok(h, h.pos, h.len - h.pos, H5_TAG_COMMENT);
            h.pos = h.len;
            h.state = HS_EOF;
            return true;
          }
          if (s[i + 1] != '>') {
            p = (uint32_t)i + 1;
            continue;
          }
          h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_TAG_COMMENT);
          h.pos = (uint32_t)i + 2;
          h.state = HS_DATA;
          return true;
        }
      }
      case HS_MARKUP_DECL_OPEN: {
        const uint32_t rem = h.len - h.pos;
        const uint8_t* p = s + h.pos;
        bool doc = rem >= 7;
        for (uint32_t k = 0; k < 7 && doc; k++) doc = li_up(p[k]) == (uint8_t)"DOCTYPE"[k];
        if (doc) { run = HS_DOCTYPE; continue; }
        bool cd = rem >= 7;
        for (uint32_t k = 0; k < 7 && cd; k++) cd = p[k] == (uint8_t)"[CDATA["[k];
        if (cd) { h.pos += 7; run = HS_CDATA; continue; }
        if (rem >= 2 && p[0] == '-' && p[1] == '-') { h.pos += 2; run = HS_COMMENT; continue; }
        run = HS_BOGUS_COMMENT;
        continue;
      }
      case HS_COMMENT: {
        uint32_t p = h.pos;
        const uint32_t n = h.len;
        while (true) {
          const int64_t i = li_memchr(s, p, n, '-');
          if (i < 0 || (int64_t)i > (int64_t)n - 3) {
            h.state = HS_EOF;
            h5_tok(h, h.pos, n - h.pos, H5_TAG_COMMENT);
            return true;
          }
          uint32_t off = 1;
          while ((uint32_t)i + off < n && s[i + off] == 0) off++;
          if ((uint32_t)i + off == n) {
            h.state = HS_EOF;
            h5_tok(h, h.pos, n - h.pos, H5_TAG_COMMENT);
            return true;
          }
          const uint8_t ch = s[i + off];
          if (ch != '-' && ch != '!') {
            p = (uint32_t)i + 1;
            continue;
          }
          off++;
          if ((uint32_t)i + off == n) {
            h.state = HS_EOF;
            h5_tok(h, h.pos, n - h.pos, H5_TAG_COMMENT);
            return true;
          }
          if (s[i + off] != '>') {
            p = (uint32_t)i + 1;
            continue;
          }
          off++;
          h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_TAG_COMMENT);
          h.pos = (uint32_t)i + off;
          h.state = HS_DATA;
          return true;
        }
      }
      case HS_CDATA: {
        uint32_t p = h.pos;
        const uint32_t n = h.len;
        while (true) {
          const int64_t i = li_memchr(s, p, n, ']');
          if (i < 0 || (int64_t)i > (int64_t)n - 3) {
            h.state = HS_EOF;
            h5_tok(h, h.pos, n - h.pos, H5_DATA_TEXT);
            return true;
          }
          if (s[i + 1] == ']' && s[i + 2] == '>') {
            h.state = HS_DATA;
            h5_tok(h, h.pos, (uint32_t)i - h.pos, H5_DATA_TEXT);
            h.pos = (uint32_t)i + 3;
            return true;
          }
          p = (uint32_t)i + 1;
        }
      }
      case HS_DOCTYPE: {
        const int64_t i = li_memchr(s, h.pos, h.len, '>');
        h.ts = h.pos;
        h.tt = H5_DOCTYPE;
        if (i < 0) {
          h.state = HS_EOF;
          h.tl = h.len - h.pos;
        } else {
          h.state = HS_DATA;
          h.tl = (uint32_t)i - h.pos;
          h.pos = (uint32_t)i + 1;
        }
        return true;
      }
      default: return false;
    }
  }
  return false;
}

// cstrcasecmp_with_null(lit, b, n) == 0: NULs in b are skipped (lit from a pool)
GI_HD bool li_eq_with_null(const uint8_t* lit, uint32_t ln, const uint8_t* b, uint32_t n) {
  uint32_t j = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t c = b[i];
    if (c == 0) continue;
    c = li_up(c);
    if (j >= ln || lit[j] != c) return false;
    j++;
  }
  return j == ln;
}

GI_HD __noinline__ bool li_black_tag(const uint8_t* s, uint32_t n) {
  if (n < 3) return false;
  for (uint32_t k = 0; k < LI_NTAGS; k++) {
    const uint32_t e = kLiTags[k];
    if (li_eq_with_null(&kLiXPool[e & 0xFFFFu], (e >> 16) & 0xFFu, s, n)) return true;
  }
  if ((s[0] == 's' || s[0] == 'S') && (s[1] == 'v' || s[1] == 'V') && (s[2] == 'g' || s[2] == 'G')) return true;
  if ((s[0] == 'x' || s[0] == 'X') && (s[1] == 's' || s[1] == 'S') && (s[2] == 'l' || s[2] == 'L')) return true;
  return false;
}

GI_HD __noinline__ uint32_t li_black_attr(const uint8_t* s, uint32_t n) {
  if (n < 2) return 0;
  if (n >= 5) {
    if ((s[0] == 'o' || s[0] == 'O') && (s[1] == 'n' || s[1] == 'N')) return 1;
    if (li_eq_with_null((const uint8_t*)"XMLNS", 5, s, 5) || li_eq_with_null((const uint8_t*)"XLINK", 5, s, 5)) return 1;
  }
  for (uint32_t k = 0; k < LI_NATTRS; k++) {
    const uint32_t e = kLiAttrs[k];
    if (li_eq_with_null(&kLiXPool[e & 0xFFFFu], (e >> 16) & 0xFFu, s, n)) return e >> 24;
  }
  return 0;
}

GI_HD __forceinline__ int li_hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return 256;
}

// html_decode_char_at over s[0, n) (bytes past n read as 0, the C NUL terminator)
GI_HD int li_html_decode_char_at(const uint8_t* s, uint32_t n, uint32_t* used) {
  auto at = [&](uint32_t k) -> uint8_t { return k < n ? s[k] : (uint8_t)0; };
  if (n == 0) {
    *used = 0;
    return -1;
  }
  *used = 1;
  if (s[0] != '&' || n < 2) return s[0];
  if (at(1) != '#') return '&';
  if (at(2) == 'x' || at(2) == 'X') {
    int ch = li_hexv(at(3));
    if (ch == 256) return '&';
    int val = ch;
    uint32_t i = 4;
    while (i < n) {
      const uint8_t c = s[i];
      if (c == ';') {
        *used = i + 1;
        return val;
      }
      ch = li_hexv(c);
      if (ch == 256) {
        *used = i;
        return val;
      }
      val = val * 16 + ch;
      if (val > 0x1000FF) return '&';
      i++;
    }
    *used = i;
    return val;
  }
  uint8_t c = at(2);
  if (c < '0' || c > '9') return '&';
  int val = c - '0';
  uint32_t i = 3;
  while (i < n) {
    c = s[i];
    if (c == ';') {
      *used = i + 1;
      return val;
    }
    if (c < '0' || c > '9') {
      *used = i;
      return val;
    }
    val = val * 10 + (c - '0');
    if (val > 0x1000FF) return '&';
    i++;
  }
  *used = i;
  return val;
}

GI_HD bool li_htmlencode_startswith(const char* prefix, const uint8_t* s, uint32_t n) {
  uint32_t j = 0;
  bool first = true;
  while (n > 0) {
    if (!prefix[j]) return true;
    uint32_t used;
    int cb = li_html_decode_char_at(s, n, &used);
    s += used;
    n -= used;
    if (first && cb <= 32) continue;
    first = false;
    if (cb == 0 || cb == 10) continue;
    if (cb >= 'a' && cb <= 'z') cb -= 0x20;
    if ((uint8_t)prefix[j] != (uint8_t)(cb & 0xFF)) return false;
    j++;
  }
  return !prefix[j];
}

GI_HD __noinline__ bool li_black_url(const uint8_t* s, uint32_t n) {
  while (n > 0 && (s[0] <= 32 || s[0] >= 127)) {
    s++;
    n--;
  }
  return li_htmlencode_startswith("DATA", s, n) || li_htmlencode_startswith("VIEW-SOURCE", s, n) ||
         li_htmlencode_startswith("JAVA", s, n) || li_htmlencode_startswith("VBSCRIPT", s, n);
}

// libinjection_is_xss for one start state
GI_HD __noinline__ bool li_xss_ctx(const uint8_t* s, uint32_t n, uint8_t start) {
  H5 h;
  h.s = s;
  h.len = n;
  h.pos = 0;
  h.ts = h.tl = 0;
  h.tt = 0xFF;
  h.is_close = 0;
  h.state = start;
  uint32_t attr = 0;
  for (uint32_t guard = 0; guard <= 4 * n + 16; guard++) {  // every token consumes input (never reached)
    if (!h5_next(h)) return false;
    const uint8_t* t = s + h.ts;
    const uint32_t tl = h.tl;
    if (h.tt != H5_ATTR_VALUE) attr = 0;
    if (h.tt == H5_DOCTYPE) return true;
    if (h.tt == H5_TAG_NAME_OPEN) {
      if (li_black_tag(t, tl)) return true;
    } else if (h.tt == H5_ATTR_NAME) {
      attr = li_black_attr(t, tl);
    } else if (h.tt == H5_ATTR_VALUE) {
      if (attr == 1 || attr == 3) return true;
      if (attr == 2 && li_black_url(t, tl)) return true;
      if (attr == 4 && li_black_attr(t, tl)) return true;
      attr = 0;
    } else if (h.tt == H5_TAG_COMMENT) {
      for (uint32_t k = 0; k < tl; k++)
        if (t[k] == '`') return true;
      if (tl > 3) {
        if (t[0] == '[' && (t[1] == 'i' || t[1] == 'I') && (t[2] == 'f' || t[2] == 'F')) return true;
        if ((t[0] == 'x' || t[0] == 'X') && (t[1] == 'm' || t[1] == 'M') && (t[2] == 'l' || t[2] == 'L')) return true;
      }
      if (tl > 5) {
        if (li_eq_with_null((const uint8_t*)"IMPORT", 6, t, 6) || li_eq_with_null((const uint8_t*)"ENTITY", 6, t, 6))
          return true;
      }
    }
  }
  return false;
}

// libinjection_xss: the five start states
GI_HD __noinline__ bool li_detect_xss(const uint8_t* s, uint32_t n) {
  return li_xss_ctx(s, n, HS_DATA) || li_xss_ctx(s, n, HS_BEFORE_ATTR_NAME) || li_xss_ctx(s, n, HS_VALUE_SQ) ||
         li_xss_ctx(s, n, HS_VALUE_DQ) || li_xss_ctx(s, n, HS_VALUE_BQ);
}

