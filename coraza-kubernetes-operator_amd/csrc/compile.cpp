// SecLang -> device rule program ("GPU artifact emitter").
//
// Replaces the compile half of coraza.NewWAF
// (/root/reference/internal/controller/ruleset_controller.go:159-160):
// [upstream coraza/v3 v3.3.3 internal/seclang/{parser,directives,rule_parser}.go]
// restated: line continuation + TrimSpace per line, directive cut at the first
// space, quoted operator via cutQuotedString (escapes kept), comma-separated
// actions with '...' quoting, SecDefaultAction merging (mergeActions), chains.
// The output is the DProgram arrays of gi_program.h plus one DFA per distinct
// @rx / @pm / @contains argument and per regex variable key.
#include "compile.h"

#include <algorithm>
#include <atomic>
#include <thread>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <sstream>
#include <unordered_map>

#include "unicode_tables.h"

namespace gi {
namespace {

const char* kWs = " \t\r\n\v\f";

std::string trim(const std::string& s, const char* set = kWs) {
  size_t a = s.find_first_not_of(set);
  if (a == std::string::npos) return "";
  size_t b = s.find_last_not_of(set);
  return s.substr(a, b - a + 1);
}
std::string lower(std::string s) {
  for (auto& c : s)
    if (c >= 'A' && c <= 'Z') c += 32;
  return s;
}
std::string upper(std::string s) {
  for (auto& c : s)
    if (c >= 'a' && c <= 'z') c -= 32;
  return s;
}
bool starts_with(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

// strconv.Atoi
bool go_atoi(const std::string& s, int64_t* v) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) {
    neg = s[i] == '-';
    i++;
  }
  if (i >= s.size()) return false;
  __int128 acc = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    acc = acc * 10 + (s[i] - '0');
    if (acc > ((__int128)1 << 64)) acc = ((__int128)1 << 64);
  }
  if (neg) acc = -acc;
  if (acc > INT64_MAX || acc < INT64_MIN) {
    *v = acc > 0 ? INT64_MAX : INT64_MIN;
    return false;
  }
  *v = (int64_t)acc;
  return true;
}

// @within over a constant argument (a literal, or TX macros the fold resolved):
// "value is a substring of arg" is a finite language; its DFA is arg's suffix
// automaton.  Stored as a byte-mode DDfa whose every state accepts except the
// last (dead, absorbing): k_eval walks the value through it -- O(len(value))
// instead of a naive substring search of the whole argument.  Returns the DFA
// id, or -1 (no automaton: the argument is too large).
int within_dfa(std::vector<DDfa>& dfas, std::vector<uint16_t>& trans, std::vector<uint8_t>& u8pool,
               const std::string& arg) {
  struct St {
    int len, link;
    int next[256];
  };
  if (arg.size() > 8000) return -1;
  std::vector<St> st;
  st.reserve(2 * arg.size() + 2);
  auto fresh = [&](int len) {
    St x;
    x.len = len;
    x.link = -1;
    for (int& n : x.next) n = -1;
    st.push_back(x);
    return (int)st.size() - 1;
  };
  fresh(0);
  int last = 0;
  for (unsigned char c : arg) {
    const int cur = fresh(st[last].len + 1);
    int p = last;
    while (p != -1 && st[p].next[c] < 0) {
      st[p].next[c] = cur;
      p = st[p].link;
    }
    if (p == -1) {
      st[cur].link = 0;
    } else {
      const int q = st[p].next[c];
      if (st[p].len + 1 == st[q].len) {
        st[cur].link = q;
      } else {
        const int clone = fresh(st[p].len + 1);
        std::copy(st[q].next, st[q].next + 256, st[clone].next);
        st[clone].link = st[q].link;
        while (p != -1 && st[p].next[c] == q) {
          st[p].next[c] = clone;
          p = st[p].link;
        }
        st[q].link = st[cur].link = clone;
      }
    }
    last = cur;
  }
  uint8_t cls[256];
  int ncls = 0;
  for (int b = 0; b < 256; b++) cls[b] = 0xFF;
  for (unsigned char c : arg)
    if (cls[c] == 0xFF) cls[c] = (uint8_t)ncls++;
  const int other = ncls++;
  for (int b = 0; b < 256; b++)
    if (cls[b] == 0xFF) cls[b] = (uint8_t)other;
  const uint32_t n = (uint32_t)st.size() + 1, dead = (uint32_t)st.size();
  if (n > 32768 || (uint64_t)n * ncls > (1u << 18)) return -1;
  DDfa h{};
  h.n_states = n;
  h.n_classes = (uint32_t)ncls;
  h.start = 0;
  h.accept = dead;  // (not a sticky accept: the dead state; only k_eval's @within walk reads this automaton)
  h.byte_mode = 1;
  h.trans_off = (uint32_t)trans.size();
  int rep[256];  // a byte of each class of the argument
  for (int b = 0; b < 256; b++)
    if (cls[b] != other) rep[cls[b]] = b;
  for (uint32_t q = 0; q < n; q++)
    for (int c = 0; c < ncls; c++) {
      const int nx = (q == dead || c == other) ? -1 : st[q].next[rep[c]];
      trans.push_back((uint16_t)(nx < 0 ? dead : (uint32_t)nx));
    }
  h.endacc_off = (uint32_t)u8pool.size();
  for (uint32_t q = 0; q < n; q++) u8pool.push_back(q == dead ? 0 : 1);
  h.amap_off = (uint32_t)u8pool.size();
  for (int b = 0; b < 256; b++) u8pool.push_back(cls[b]);
  dfas.push_back(h);
  return (int)dfas.size() - 1;
}

struct CompileError {
  int code;
  std::string msg;
};
[[noreturn]] void perr(const std::string& m) { throw CompileError{-1, m}; }
[[noreturn]] void unsup(const std::string& m) { throw CompileError{-2, m}; }

// ------------------------------------------------------------------- IR
struct IrVar {
  std::string name;
  std::string key;
  bool key_rx = false;
  bool count = false;
  std::vector<std::pair<std::string, bool>> exc;  // (lowercased key | regex source, is_rx)
};
struct IrNd {  // non-disruptive action in order
  bool is_setvar;
  std::string sv_key, sv_value;
  bool sv_remove = false;
  std::string ctl_name, ctl_value;
};
struct IrRule {
  int id = 0, phase = 2, line = 0;
  std::vector<std::string> tags;  // tag:'...' values (SecRuleRemoveByTag, ctl:ruleRemove*ByTag)
  std::string msg;                // msg:'...' as written (SecRuleRemoveByMsg, ctl:ruleRemove*ByMsg)
  // a construct coraza.NewWAF accepts that this engine does not evaluate (a
  // RESPONSE_* variable, an operator / transformation / ctl of the response
  // path): harmless in a phase 3-5 rule (never evaluated by the request path),
  // GI_EUNSUPPORTED in a phase 1-2 rule
  std::string deferred;
  std::vector<IrVar> vars;
  bool has_op = false;
  std::string op_name, op_arg;
  bool op_neg = false;
  std::vector<std::string> transforms;
  std::string disruptive;
  int status = 0;
  bool capture = false, multimatch = false;
  std::vector<std::string> phrases;  // @pmFromFile: the data file's phrases (lowercased)
  std::vector<IrNd> nd;
  int skip = 0;
  std::string skip_after, secmark;
  bool has_chain = false;
  std::vector<IrRule> children;  // only on chain starters
};
using Actions = std::vector<std::pair<std::string, std::string>>;
struct IrWaf {
  std::string engine = "On";
  int64_t args_limit = 1000;  // SecArgumentsLimit (coraza WAF.ArgumentLimit)
  bool body_access = false;
  int64_t body_limit = 134217728;
  bool body_partial = false;
  std::vector<IrRule> rules;
  std::map<int, Actions> defaults;
};

const std::map<std::string, std::string>& action_types() {
  static const std::map<std::string, std::string> t = {
      {"deny", "disruptive"}, {"drop", "disruptive"}, {"pass", "disruptive"},
      {"block", "disruptive"}, {"redirect", "disruptive"}, {"allow", "disruptive"},
      {"chain", "flow"}, {"skip", "flow"}, {"skipafter", "flow"},
      {"id", "metadata"}, {"phase", "metadata"}, {"msg", "metadata"}, {"tag", "metadata"},
      {"severity", "metadata"}, {"ver", "metadata"}, {"rev", "metadata"},
      {"maturity", "metadata"}, {"accuracy", "metadata"},
      {"status", "data"}, {"xmlns", "data"},
      {"t", "nondisruptive"}, {"setvar", "nondisruptive"}, {"capture", "nondisruptive"},
      {"log", "nondisruptive"}, {"nolog", "nondisruptive"}, {"auditlog", "nondisruptive"},
      {"noauditlog", "nondisruptive"}, {"logdata", "nondisruptive"},
      {"multimatch", "nondisruptive"}, {"ctl", "nondisruptive"},
      {"expirevar", "nondisruptive"}, {"initcol", "nondisruptive"},
      {"sanitisearg", "nondisruptive"}, {"sanitisematched", "nondisruptive"},
      {"setenv", "nondisruptive"}, {"append", "nondisruptive"},
      {"sanitiserequestheader", "nondisruptive"}, {"sanitiseresponseheader", "nondisruptive"},
  };
  return t;
}

bool ignored_directive(const std::string& d) {
  static const char* ign[] = {
      "secresponsebodyaccess", "secresponsebodymimetype", "secresponsebodylimit",
      "secresponsebodylimitaction", "secauditengine", "secauditlogtype", "secauditlog",
      "secauditlogformat", "secauditlogparts", "secauditlogrelevantstatus",
      "secauditlogstoragedir", "secauditlogdirmode", "secauditlogfilemode", "secdebuglog",
      "secdebugloglevel", "seccomponentsignature", "secrequestbodyinmemorylimit", "sectmpdir",
      "secdatadir", "secargumentseparator", "seccollectiontimeout", "secrequestbodynofileslimit",
      "secuploaddir", "secuploadkeepfiles", "secuploadfilemode", "secunicodemap",
      "secpcrematchlimit", "secpcrematchlimitrecursion", "secstatusengine", "secconnengine",
      "secserversignature", "sechttpblkey", "secwebappid", "secsensorid",
      "secrequestbodyjsondepthlimit", "secresponsebodymimetypesclear", "seccookieformat",
      "secuploadfilelimit", "secignorerulecompilationerrors"};
  for (auto* s : ign)
    if (d == s) return true;
  return starts_with(d, "secaudit") || starts_with(d, "secdebug");
}

int parse_phase(const std::string& v) {
  std::string l = lower(v);
  if (l == "request") return 2;
  if (l == "response") return 4;
  if (l == "logging") return 5;
  int64_t p;
  if (!go_atoi(v, &p) || p < 1 || p > 5) perr("invalid phase " + v);
  return (int)p;
}

Actions parse_actions(const std::string& s) {
  std::vector<std::string> items;
  std::string cur;
  bool quote = false;
  for (char ch : s) {
    if (ch == '\'') {
      quote = !quote;
      cur += ch;
      continue;
    }
    if (ch == ',' && !quote) {
      items.push_back(cur);
      cur.clear();
      continue;
    }
    cur += ch;
  }
  if (!trim(cur).empty()) items.push_back(cur);
  Actions res;
  for (auto& it : items) {
    std::string item = trim(it);
    if (item.empty()) continue;
    std::string k, v;
    size_t c = item.find(':');
    if (c == std::string::npos) {
      k = item;
    } else {
      k = item.substr(0, c);
      v = item.substr(c + 1);
    }
    k = lower(trim(k));
    v = trim(v);
    if (v.size() >= 2 && v.front() == '\'' && v.back() == '\'') v = v.substr(1, v.size() - 2);
    if (!action_types().count(k)) perr("unknown action " + k);
    res.push_back({k, v});
  }
  return res;
}

std::pair<std::string, std::string> cut_quoted(const std::string& s) {
  if (s.empty() || s[0] != '"') perr("expected quoted string: " + s);
  for (size_t i = 1; i < s.size(); i++) {
    if (s[i] != '"') continue;
    if (s[i - 1] == '\\') continue;
    return {s.substr(1, i - 1), s.substr(i + 1)};
  }
  perr("expected terminating quote: " + s);
}

const std::vector<std::string>& single_names() {
  static const std::vector<std::string> v = {
      "REQUEST_METHOD", "REQUEST_PROTOCOL", "REQUEST_URI", "REQUEST_URI_RAW", "REQUEST_LINE",
      "REQUEST_FILENAME", "REQUEST_BASENAME", "QUERY_STRING", "REQUEST_BODY",
      "REQUEST_BODY_LENGTH", "REQBODY_ERROR", "REQBODY_ERROR_MSG", "REQBODY_PROCESSOR",
      "MULTIPART_STRICT_ERROR", "REMOTE_ADDR", "REMOTE_PORT", "FILES_COMBINED_SIZE", "ARGS_COMBINED_SIZE",
      "FULL_REQUEST_LENGTH", "URLENCODED_ERROR", "INBOUND_DATA_ERROR", "SERVER_NAME"};
  return v;
}
const std::map<std::string, int>& collection_ids() {
  static const std::map<std::string, int> m = {
      {"ARGS_GET", V_ARGS_GET}, {"ARGS_POST", V_ARGS_POST}, {"ARGS", V_ARGS},
      {"REQUEST_HEADERS", V_REQUEST_HEADERS}, {"REQUEST_COOKIES", V_REQUEST_COOKIES},
      {"TX", V_TX}, {"ARGS_GET_NAMES", V_ARGS_GET_NAMES}, {"ARGS_POST_NAMES", V_ARGS_POST_NAMES},
      {"ARGS_NAMES", V_ARGS_NAMES}, {"REQUEST_HEADERS_NAMES", V_REQUEST_HEADERS_NAMES},
      {"REQUEST_COOKIES_NAMES", V_REQUEST_COOKIES_NAMES}, {"XML", V_XML}, {"FILES", V_FILES},
      {"FILES_NAMES", V_FILES_NAMES}, {"FILES_SIZES", V_FILES_SIZES}, {"FILES_TMPNAMES", V_FILES_TMPNAMES},
      {"MULTIPART_PART_HEADERS", V_MULTIPART_PART_HEADERS},
      {"MATCHED_VAR", V_MATCHED_VAR}, {"MATCHED_VAR_NAME", V_MATCHED_VAR_NAME},
      {"MATCHED_VARS", V_MATCHED_VARS}, {"MATCHED_VARS_NAMES", V_MATCHED_VARS_NAMES}};
  return m;
}
// Variables coraza v3.3.3 declares [upstream internal/variables/variables.go]
// that the request path does not evaluate: the response phases' variables
// (RESPONSE-950..980 read RESPONSE_BODY / RESPONSE_STATUS / RESPONSE_HEADERS),
// and a few request-side ones this engine has no value for.  The parser
// accepts them, as NewWAF does; a phase 1-2 rule that reads one is
// GI_EUNSUPPORTED (IrRule::deferred).
bool known_unsupported_var(const std::string& n) {
  static const char* u[] = {
      "RESPONSE_BODY", "RESPONSE_STATUS", "RESPONSE_HEADERS", "RESPONSE_HEADERS_NAMES", "RESPONSE_PROTOCOL",
      "RESPONSE_CONTENT_TYPE", "RESPONSE_CONTENT_LENGTH", "RESPONSE_ARGS", "RESPONSE_XML", "RES_BODY_PROCESSOR",
      "OUTBOUND_DATA_ERROR", "STATUS_LINE", "SERVER_ADDR", "SERVER_PORT", "UNIQUE_ID", "REMOTE_HOST",
      "HIGHEST_SEVERITY", "DURATION", "REQBODY_PROCESSOR_ERROR", "REQBODY_PROCESSOR_ERROR_MSG", "ARGS_PATH",
      "FILES_TMP_CONTENT", "MULTIPART_FILENAME", "MULTIPART_NAME", "MULTIPART_DATA_AFTER", "GEO", "RULE", "JSON",
      "ENV", "REQUEST_XML", "AUTH_TYPE", "TIME", "TIME_DAY", "TIME_EPOCH", "TIME_HOUR", "TIME_MIN", "TIME_MON",
      "TIME_SEC", "TIME_WDAY", "TIME_YEAR"};
  for (auto* s : u)
    if (n == s) return true;
  return false;
}
int single_id(const std::string& n) {
  auto& v = single_names();
  for (size_t i = 0; i < v.size(); i++)
    if (v[i] == n) return (int)i;
  return -1;
}
bool is_known_var(const std::string& n) {
  return single_id(n) >= 0 || collection_ids().count(n) || known_unsupported_var(n);
}

void parse_variables(const std::string& s, IrRule* rule) {
  std::vector<std::string> parts;
  std::string cur;
  bool in_rx = false;
  for (size_t i = 0; i < s.size(); i++) {
    char ch = s[i];
    if (ch == '/' && !cur.empty() && cur.back() == ':' && !in_rx) {
      in_rx = true;
      cur += ch;
    } else if (ch == '/' && in_rx) {
      in_rx = false;
      cur += ch;
    } else if (ch == '|' && !in_rx) {
      parts.push_back(cur);
      cur.clear();
    } else {
      cur += ch;
    }
  }
  parts.push_back(cur);
  for (auto p : parts) {
    p = trim(p);
    if (p.empty()) continue;
    bool neg = false, cnt = false;
    if (p[0] == '!') {
      neg = true;
      p = p.substr(1);
    } else if (p[0] == '&') {
      cnt = true;
      p = p.substr(1);
    }
    std::string name, key;
    size_t c = p.find(':');
    if (c == std::string::npos) {
      name = p;
    } else {
      name = p.substr(0, c);
      key = p.substr(c + 1);
    }
    name = upper(name);
    if (!is_known_var(name)) perr("unknown variable " + name);
    if (known_unsupported_var(name) && rule->deferred.empty()) rule->deferred = "unsupported variable " + name;
    bool key_rx = false;
    if (key.size() >= 2 && key.front() == '\'' && key.back() == '\'') key = key.substr(1, key.size() - 2);
    if (key.size() > 2 && key.front() == '/' && key.back() == '/') {
      key = key.substr(1, key.size() - 2);
      key_rx = true;
      Regex re;
      std::string err;
      if (!re_parse(key, &re, &err)) perr("invalid key regex /" + key + "/: " + err);
    }
    if (neg) {
      bool matched = false;
      for (auto& rv : rule->vars)
        if (rv.name == name) {
          rv.exc.push_back({key_rx ? key : lower(key), key_rx});
          matched = true;
        }
      if (!matched) perr("cannot negate variable " + name + " that is not targeted");
      continue;
    }
    if (single_id(name) >= 0 && !key.empty()) perr("variable " + name + " does not accept a key");
    IrVar v;
    v.name = name;
    v.key = key;
    v.key_rx = key_rx;
    v.count = cnt;
    rule->vars.push_back(v);
  }
}

// @pmFromFile data files of the compile in progress (compile_program).
thread_local const std::map<std::string, std::string>* g_data_files = nullptr;

// coraza internal/operators/pm_from_file.go: bufio.Scanner lines ('\n', a
// trailing '\r' dropped), strings.TrimSpace, empty lines and '#' comments
// skipped, strings.ToLower; then the same ASCII case-insensitive
// aho-corasick matcher as @pm.
std::vector<std::string> pm_file_phrases(const std::string& data, bool lowered = true) {
  std::vector<std::string> out;
  size_t pos = 0;
  while (pos < data.size()) {
    size_t nl = data.find('\n', pos);
    if (nl == std::string::npos) nl = data.size();
    std::string l = data.substr(pos, nl - pos);
    pos = nl + 1;
    if (!l.empty() && l.back() == '\r') l.pop_back();
    l = trim(l);
    if (l.empty() || l[0] == '#') continue;
    out.push_back(lowered ? lower(l) : l);
  }
  return out;
}

// Go net.ParseIP (no zone; IPv4 fields without leading zeros): 4 or 16 bytes
// in `out` (n = 4 for IPv4, 16 for IPv6).  [Go net/netip parse rules]
bool go_parse_ipv4(const std::string& s, uint8_t out[4]) {
  size_t i = 0;
  for (int f = 0; f < 4; f++) {
    if (f) {
      if (i >= s.size() || s[i] != '.') return false;
      i++;
    }
    size_t j = i;
    int v = 0;
    while (j < s.size() && j - i < 3 && s[j] >= '0' && s[j] <= '9') v = v * 10 + (s[j++] - '0');
    if (j == i || v > 255 || (j - i > 1 && s[i] == '0')) return false;
    out[f] = (uint8_t)v;
    i = j;
  }
  return i == s.size();
}
bool go_parse_ip(const std::string& s, uint8_t out[16], int* n) {
  if (s.find(':') == std::string::npos) {
    *n = 4;
    return go_parse_ipv4(s, out);
  }
  if (s.find('%') != std::string::npos) return false;
  *n = 16;
  uint16_t g[8] = {0};
  int ng = 0, gap = -1;
  size_t i = 0;
  if (s.compare(0, 2, "::") == 0) {
    gap = 0;
    i = 2;
    if (i == s.size()) {
      memset(out, 0, 16);
      return true;
    }
  }
  while (i < s.size()) {
    if (ng == 8) return false;
    size_t j = i;
    uint32_t v = 0;
    while (j < s.size() && j - i < 4 && isxdigit((unsigned char)s[j])) {
      const char c = (char)tolower((unsigned char)s[j]);
      v = v * 16 + (c <= '9' ? c - '0' : c - 'a' + 10);
      j++;
    }
    if (j < s.size() && s[j] == '.') {  // embedded IPv4 in the last 32 bits
      uint8_t v4[4];
      if (ng > 6 || !go_parse_ipv4(s.substr(i), v4)) return false;
      g[ng++] = (uint16_t)(v4[0] << 8 | v4[1]);
      g[ng++] = (uint16_t)(v4[2] << 8 | v4[3]);
      i = s.size();
      break;
    }
    if (j == i) return false;
    g[ng++] = (uint16_t)v;
    i = j;
    if (i == s.size()) break;
    if (s[i] != ':') return false;
    i++;
    if (i < s.size() && s[i] == ':') {
      if (gap >= 0) return false;
      gap = ng;
      i++;
      if (i == s.size()) break;
    } else if (i == s.size()) {
      return false;
    }
  }
  if (gap < 0 && ng != 8) return false;
  if (gap >= 0 && ng > 7) return false;
  uint16_t full[8] = {0};
  if (gap < 0) {
    memcpy(full, g, sizeof(full));
  } else {
    for (int k = 0; k < gap; k++) full[k] = g[k];
    const int tail = ng - gap;
    for (int k = 0; k < tail; k++) full[8 - tail + k] = g[gap + k];
  }
  for (int k = 0; k < 8; k++) {
    out[2 * k] = (uint8_t)(full[k] >> 8);
    out[2 * k + 1] = (uint8_t)full[k];
  }
  return true;
}

// coraza ipmatch.go: comma-separated networks; a bare address is /32 or /128;
// net.ParseCIDR (the address is masked to the prefix); entries that do not
// parse are skipped.  Records: GI_IPNET_BYTES each.
std::string ipmatch_records(const std::string& arg, size_t* count) {
  std::string out;
  *count = 0;
  size_t pos = 0;
  while (pos <= arg.size()) {
    size_t c = arg.find(',', pos);
    if (c == std::string::npos) c = arg.size();
    std::string e = trim(arg.substr(pos, c - pos));
    pos = c + 1;
    if (e.empty()) continue;
    std::string addr = e;
    int bits = -1;
    size_t sl = e.find('/');
    if (sl != std::string::npos) {
      addr = e.substr(0, sl);
      const std::string b = e.substr(sl + 1);
      // net.ParseCIDR reads the prefix with dtoi (decimal digits, leading zeros allowed)
      if (b.empty() || b.size() > 8 || b.find_first_not_of("0123456789") != std::string::npos) continue;
      bits = atoi(b.c_str());
    }
    uint8_t ip[16];
    int n = 0;
    if (!go_parse_ip(addr, ip, &n)) continue;
    if (bits < 0) bits = n == 4 ? 32 : 128;
    if (bits > 8 * n) continue;
    for (int k = 0; k < n; k++) {
      const int keep = std::min(8, std::max(0, bits - 8 * k));
      ip[k] &= (uint8_t)(keep == 8 ? 0xFF : (0xFF00 >> keep) & 0xFF);
    }
    // IPNet.Contains works on To4() of the network number: a (masked)
    // IPv4-mapped IPv6 network is an IPv4 network with the mask's low 32 bits
    if (n == 16 && ip[10] == 0xFF && ip[11] == 0xFF && !ip[0] && !ip[1] && !ip[2] && !ip[3] && !ip[4] && !ip[5] &&
        !ip[6] && !ip[7] && !ip[8] && !ip[9]) {
      memmove(ip, ip + 12, 4);
      n = 4;
      bits = std::max(0, bits - 96);
    }
    std::string rec(GI_IPNET_BYTES, '\0');
    rec[0] = (char)n;
    rec[1] = (char)bits;
    for (int k = 0; k < n; k++) rec[2 + k] = (char)ip[k];
    out += rec;
    (*count)++;
  }
  return out;
}

void parse_operator(std::string opstr, IrRule* rule) {
  if (opstr.empty() || (opstr[0] != '@' && (opstr.size() < 2 || opstr[1] != '@'))) opstr = "@rx " + opstr;
  std::string raw, data;
  size_t sp = opstr.find(' ');
  if (sp == std::string::npos) {
    raw = opstr;
  } else {
    raw = opstr.substr(0, sp);
    data = opstr.substr(sp + 1);
  }
  raw = trim(raw);
  data = trim(data);
  std::string name;
  if (starts_with(raw, "!@")) {
    rule->op_neg = true;
    name = raw.substr(2);
  } else if (starts_with(raw, "@")) {
    name = raw.substr(1);
  } else {
    name = raw;
  }
  rule->has_op = true;
  rule->op_name = lower(name);
  rule->op_arg = data;
  static const char* known[] = {"rx", "pm", "contains", "containsword", "streq", "beginswith",
                                "endswith", "within", "eq", "ge", "gt", "le", "lt",
                                "unconditionalmatch", "nomatch", "validatebyterange",
                                "validateurlencoding", "validateutf8encoding", "pmfromfile", "ipmatch",
                                "ipmatchfromfile", "ipmatchf", "detectsqli", "detectxss"};
  // operators coraza v3.3.3 has [upstream internal/operators] that this engine does not evaluate
  static const char* later[] = {"geolookup", "inspectfile", "pmfromdataset", "ipmatchfromdataset", "rbl",
                                "restpath", "strmatch", "validatenid", "validateschema", "verifycc",
                                "verifycpf", "verifyssn", "fuzzyhash"};
  bool ok = false;
  for (auto* k : known)
    if (rule->op_name == k) ok = true;
  if (!ok) {
    for (auto* k : later)
      if (rule->op_name == k) {
        if (rule->deferred.empty()) rule->deferred = "unsupported operator @" + name;
        return;
      }
    perr("invalid operator @" + name);
  }
  if (rule->op_name == "pmfromfile") {
    if (!g_data_files || !g_data_files->count(data)) perr("open " + data + ": no such file or directory");
    rule->phrases = pm_file_phrases(g_data_files->at(data));
  }
  if (rule->op_name == "ipmatchfromfile" || rule->op_name == "ipmatchf") {
    // ipmatchfromfile.go: one network per line (comments and blank lines skipped)
    if (!g_data_files || !g_data_files->count(data)) perr("open " + data + ": no such file or directory");
    std::string list;
    for (const auto& p : pm_file_phrases(g_data_files->at(data), false)) list.append(p).push_back(',');
    rule->op_name = "ipmatch";
    rule->op_arg = list;
  }
  if (rule->op_name == "rx") {
    Regex re;
    std::string err;
    if (!re_parse("(?sm)" + data, &re, &err)) perr("invalid regex " + data + ": " + err);
  }
}

bool transform_code(const std::string& t, uint8_t* code) {
  static const std::map<std::string, uint8_t> m = {
      {"lowercase", T_LOWERCASE}, {"urldecode", T_URLDECODE}, {"urldecodeuni", T_URLDECODEUNI},
      {"htmlentitydecode", T_HTMLENTITYDECODE}, {"removenulls", T_REMOVENULLS},
      {"replacenulls", T_REPLACENULLS}, {"removewhitespace", T_REMOVEWHITESPACE},
      {"compresswhitespace", T_COMPRESSWHITESPACE}, {"replacecomments", T_REPLACECOMMENTS},
      {"cmdline", T_CMDLINE}, {"length", T_LENGTH}, {"trim", T_TRIM}, {"trimleft", T_TRIMLEFT},
      {"trimright", T_TRIMRIGHT}, {"normalizepath", T_NORMALIZEPATH},
      {"normalisepath", T_NORMALIZEPATH}, {"normalizepathwin", T_NORMALIZEPATHWIN},
      {"normalisepathwin", T_NORMALIZEPATHWIN}, {"jsdecode", T_JSDECODE},
      {"utf8tounicode", T_UTF8TOUNICODE}, {"base64decode", T_BASE64DECODE},
      {"base64decodeext", T_BASE64DECODEEXT}, {"base64encode", T_BASE64ENCODE}, {"hexdecode", T_HEXDECODE},
      {"hexencode", T_HEXENCODE}, {"sha1", T_SHA1}, {"md5", T_MD5}, {"urlencode", T_URLENCODE},
      {"cssdecode", T_CSSDECODE}, {"escapeseqdecode", T_ESCAPESEQDECODE},
      {"removecommentschar", T_REMOVECOMMENTSCHAR}};
  auto it = m.find(t);
  if (it == m.end()) return false;
  *code = it->second;
  return true;
}

void apply_actions(IrRule* rule, const Actions& acts) {
  for (auto& kv : acts) {
    const std::string& k = kv.first;
    const std::string& v = kv.second;
    if (k == "id") {
      int64_t id;
      if (!go_atoi(v, &id)) perr("invalid rule id " + v);
      rule->id = (int)id;
    } else if (k == "phase") {
      rule->phase = parse_phase(v);
    } else if (k == "deny" || k == "drop" || k == "pass" || k == "block" || k == "redirect" ||
               k == "allow") {
      rule->disruptive = k;
      if (k == "allow") {
        // [upstream internal/actions/allow.go Init]: "" every phase, "phase", "request"
        const std::string a = lower(v);
        if (a.empty()) rule->disruptive = "allow";
        else if (a == "phase") rule->disruptive = "allow:phase";
        else if (a == "request") rule->disruptive = "allow:request";
        else perr("invalid argument " + v + " for allow");
      }
    } else if (k == "tag") {
      rule->tags.push_back(v);
    } else if (k == "msg") {
      rule->msg = v;
    } else if (k == "status") {
      int64_t st;
      if (!go_atoi(v, &st)) perr("invalid status " + v);
      rule->status = (int)st;
    } else if (k == "chain") {
      rule->has_chain = true;
    } else if (k == "skip") {
      int64_t n;
      if (!go_atoi(v, &n)) perr("invalid skip " + v);
      rule->skip = (int)n;
    } else if (k == "skipafter") {
      rule->skip_after = v;
    } else if (k == "t") {
      std::string tl = lower(v);
      if (tl == "none") {
        rule->transforms.clear();
      } else {
        uint8_t code;
        if (!transform_code(tl, &code)) {
          // coraza v3.3.3's other transformations [upstream internal/transformations]
          if (tl == "removecomments" || tl == "sqlhexdecode" || tl == "uppercase") {
            if (rule->deferred.empty()) rule->deferred = "unsupported transformation t:" + v;
            continue;
          }
          perr("invalid transformation t:" + v);
        }
        rule->transforms.push_back(tl);
      }
    } else if (k == "capture") {
      rule->capture = true;
    } else if (k == "multimatch") {
      rule->multimatch = true;
    } else if (k == "setvar") {
      IrNd nd;
      nd.is_setvar = true;
      std::string s = v;
      if (!s.empty() && s[0] == '!') {
        nd.sv_remove = true;
        s = s.substr(1);
      }
      size_t dot = s.find('.');
      std::string col = dot == std::string::npos ? s : s.substr(0, dot);
      if (lower(trim(col)) != "tx") unsup("setvar only supports the TX collection");
      std::string rest = dot == std::string::npos ? "" : s.substr(dot + 1);
      if (nd.sv_remove) {
        nd.sv_key = trim(rest);
      } else {
        size_t eq = rest.find('=');
        nd.sv_key = trim(eq == std::string::npos ? rest : rest.substr(0, eq));
        nd.sv_value = eq == std::string::npos ? "" : rest.substr(eq + 1);
      }
      rule->nd.push_back(nd);
    } else if (k == "ctl") {
      IrNd nd;
      nd.is_setvar = false;
      size_t eq = v.find('=');
      nd.ctl_name = lower(trim(eq == std::string::npos ? v : v.substr(0, eq)));
      nd.ctl_value = trim(eq == std::string::npos ? "" : v.substr(eq + 1));
      // [upstream internal/actions/ctl.go]: the ctl options coraza v3.3.3 parses
      static const char* evaluated[] = {"ruleremovebyid", "ruleremovetargetbyid", "ruleremovebytag",
                                        "ruleremovetargetbytag", "ruleremovebymsg", "ruleremovetargetbymsg",
                                        "ruleengine", "requestbodyprocessor", "requestbodyaccess",
                                        "forcerequestbodyvariable"};
      // audit / debug logging and the response body: no effect on a request-phase verdict
      static const char* no_effect[] = {"auditengine", "auditlogparts", "debugloglevel", "responsebodyaccess",
                                        "responsebodylimit", "responsebodyprocessor", "forceresponsebodyvariable",
                                        "hashengine", "hashenforcement"};
      bool known = false;
      for (auto* c : evaluated) known = known || nd.ctl_name == c;
      if (!known) {
        bool ign = false;
        for (auto* c : no_effect) ign = ign || nd.ctl_name == c;
        if (ign) continue;
        if (nd.ctl_name == "requestbodylimit") {
          if (rule->deferred.empty()) rule->deferred = "unsupported ctl " + nd.ctl_name;
          continue;
        }
        perr("unknown ctl " + nd.ctl_name);
      }
      rule->nd.push_back(nd);
    }
  }
}

Actions merge_defaults(const Actions& acts, const Actions& defs) {
  Actions res;
  std::pair<std::string, std::string> da;
  bool have_da = false;
  for (auto& kv : defs) {
    const std::string& t = action_types().at(kv.first);
    if (t == "disruptive") {
      da = kv;
      have_da = true;
      continue;
    }
    if (t == "metadata") continue;
    res.push_back(kv);
  }
  bool has_block = false;
  for (auto& kv : acts) {
    if (kv.first == "block") has_block = true;
    res.push_back(kv);
  }
  if (has_block && have_da) res.push_back(da);
  return res;
}

// id or "lo-hi" (coraza directives.go / ctl.go rangeToInts)
bool parse_id_range(const std::string& s, int64_t* lo, int64_t* hi) {
  const size_t dash = s.find('-', 1);
  if (dash == std::string::npos) {
    if (!go_atoi(s, lo)) return false;
    *hi = *lo;
    return true;
  }
  return go_atoi(s.substr(0, dash), lo) && go_atoi(s.substr(dash + 1), hi);
}

IrWaf parse_seclang(const std::string& text) {
  IrWaf waf;
  // top-level rule ids in the group (coraza RuleGroup.Add rejects a repeated
  // non-zero id: "there is a another rule with id"); removal frees an id
  std::map<int, int> id_count;
  auto erase_rules = [&](const std::function<bool(const IrRule&)>& pred) {
    std::vector<IrRule> kept;
    kept.reserve(waf.rules.size());
    for (auto& r : waf.rules) {
      if (pred(r)) {
        if (r.id != 0 && --id_count[r.id] == 0) id_count.erase(r.id);
      } else {
        kept.push_back(std::move(r));
      }
    }
    waf.rules.swap(kept);
  };
  auto has_tag = [](const IrRule& r, const std::string& t) {
    return std::find(r.tags.begin(), r.tags.end(), t) != r.tags.end();
  };
  auto strip_q = [](const std::string& x) { return trim(trim(x), "\""); };
  std::vector<std::pair<int, std::string>> lines;
  {
    std::string buf;
    int lineno = 0, start = 0;
    size_t pos = 0;
    while (pos <= text.size()) {
      size_t nl = text.find('\n', pos);
      if (nl == std::string::npos) nl = text.size();
      std::string raw = text.substr(pos, nl - pos);
      lineno++;
      std::string line = trim(raw);
      if (buf.empty()) start = lineno;
      if (!line.empty() && line.back() == '\\') {
        buf += line.substr(0, line.size() - 1);
      } else {
        buf += line;
        lines.push_back({start, buf});
        buf.clear();
      }
      pos = nl + 1;
    }
    if (!buf.empty()) lines.push_back({start, buf});
  }
  IrRule* parent = nullptr;  // open chain starter (in waf.rules)
  for (auto& ln : lines) {
    const std::string& line = ln.second;
    if (line.empty() || line[0] == '#') continue;
    size_t sp = line.find(' ');
    std::string directive = sp == std::string::npos ? line : line.substr(0, sp);
    std::string opts = sp == std::string::npos ? "" : line.substr(sp + 1);
    if (opts.size() >= 3 && opts.front() == '"' && opts.back() == '"') opts = trim(opts, "\"");
    std::string d = lower(directive);
    if (d == "secruleengine") {
      std::string o = lower(trim(opts));
      if (o == "on") waf.engine = "On";
      else if (o == "off") waf.engine = "Off";
      else if (o == "detectiononly") waf.engine = "DetectionOnly";
      else perr("invalid SecRuleEngine " + opts);
    } else if (d == "secrequestbodyaccess") {
      waf.body_access = lower(trim(opts)) == "on";
    } else if (d == "secrequestbodylimit") {
      int64_t v;
      if (!go_atoi(trim(opts), &v)) perr("invalid SecRequestBodyLimit");
      waf.body_limit = v;
    } else if (d == "secrequestbodylimitaction") {
      const std::string o = lower(trim(opts));
      if (o == "processpartial") waf.body_partial = true;
      else if (o == "reject") waf.body_partial = false;
      else perr("invalid SecRequestBodyLimitAction " + opts);
    } else if (d == "secargumentslimit") {
      int64_t v;
      if (!go_atoi(trim(opts), &v)) perr("syntax error: SecArgumentsLimit [POSITIVE_INT]");
      waf.args_limit = v;
    } else if (d == "secruleremovebyid" || d == "secruleremovebytag" || d == "secruleremovebymsg") {
      // [upstream internal/seclang/directives.go directiveSecRuleRemoveBy{ID,Tag,Msg}]:
      // the rules defined so far leave the group (a chain goes with its parent)
      if (parent) perr(directive + " inside a chain");
      if (trim(opts).empty()) perr("expected options for " + directive);
      if (d == "secruleremovebyid") {
        std::stringstream ss(opts);
        std::string part;
        while (ss >> part) {
          int64_t lo, hi;
          if (!parse_id_range(part, &lo, &hi)) perr("invalid id " + part + " for SecRuleRemoveById");
          erase_rules([&](const IrRule& r) { return r.id >= lo && r.id <= hi; });
        }
      } else if (d == "secruleremovebytag") {
        const std::string tag = strip_q(opts);
        erase_rules([&](const IrRule& r) { return has_tag(r, tag); });
      } else {
        const std::string msg = strip_q(opts);
        erase_rules([&](const IrRule& r) { return r.secmark.empty() && r.msg == msg; });
      }
    } else if (d == "secruleupdatetargetbyid" || d == "secruleupdatetargetbytag" ||
               d == "secruleupdatetargetbymsg" || d == "secruleupdateactionbyid") {
      // [upstream directives.go directiveSecRuleUpdate{Target,Action}By*]: the
      // variables (negations add exceptions to the rule's existing targets) or
      // actions are parsed into the matching rules defined so far
      if (parent) perr(directive + " inside a chain");
      const std::string o = trim(opts);
      const size_t sp2 = o.find(' ');
      if (sp2 == std::string::npos) perr("syntax error: " + directive + " <selector> \"...\"");
      const std::string sel = strip_q(o.substr(0, sp2)), arg = strip_q(o.substr(sp2 + 1));
      std::vector<IrRule*> hit;
      int64_t lo = 0, hi = -1;
      if (d == "secruleupdatetargetbyid" || d == "secruleupdateactionbyid") {
        if (!parse_id_range(sel, &lo, &hi)) perr("invalid id " + sel + " for " + directive);
      }
      for (auto& r : waf.rules) {
        if (!r.secmark.empty()) continue;
        const bool m = d == "secruleupdatetargetbytag" ? has_tag(r, sel)
                       : d == "secruleupdatetargetbymsg" ? r.msg == sel
                                                         : (r.id >= lo && r.id <= hi);
        if (m) hit.push_back(&r);
      }
      if ((d == "secruleupdatetargetbyid" || d == "secruleupdateactionbyid") && lo == hi && hit.empty())
        perr(directive + ": rule \"" + sel + "\" not found");
      for (IrRule* r : hit) {
        if (d == "secruleupdateactionbyid") {
          const Actions acts = parse_actions(arg);
          bool disr = false;
          for (auto& kv : acts) {
            if (kv.first == "id" || kv.first == "chain") perr("SecRuleUpdateActionById: action " + kv.first + " cannot be updated");
            disr = disr || action_types().at(kv.first) == "disruptive";
          }
          if (disr) r->disruptive.clear();  // [upstream] Rule.ClearDisruptiveActions
          apply_actions(r, acts);
          for (auto& c : r->children) c.phase = r->phase;
        } else {
          parse_variables(arg, r);
        }
      }
    } else if (d == "secdefaultaction") {
      Actions acts = parse_actions(opts);
      int phase = 2;
      for (auto& kv : acts)
        if (kv.first == "phase") phase = parse_phase(kv.second);
      waf.defaults[phase] = acts;
    } else if (d == "secmarker") {
      if (parent) perr("SecMarker inside a chain");
      IrRule r;
      r.phase = 0;
      r.line = ln.first;
      r.secmark = trim(trim(opts), "\"");
      waf.rules.push_back(r);
    } else if (d == "secrule" || d == "secaction") {
      IrRule rule;
      rule.line = ln.first;
      std::string acts_s;
      if (d == "secrule") {
        std::string rest = trim(opts, " \t");
        std::string vars_s;
        if (!rest.empty() && rest[0] == '"') {
          auto q = cut_quoted(rest);
          vars_s = q.first;
          rest = q.second;
        } else {
          size_t s2 = rest.find(' ');
          vars_s = s2 == std::string::npos ? rest : rest.substr(0, s2);
          rest = s2 == std::string::npos ? "" : rest.substr(s2 + 1);
        }
        parse_variables(vars_s, &rule);
        rest = trim(rest);
        auto q = cut_quoted(rest);
        parse_operator(q.first, &rule);
        rest = trim(q.second);
        acts_s = rest.empty() ? "" : trim(rest, "\"");
      } else {
        acts_s = opts;
      }
      Actions acts = acts_s.empty() ? Actions() : parse_actions(acts_s);
      bool is_child = parent != nullptr;
      if (!is_child) {
        int phase = 2;
        for (auto& kv : acts)
          if (kv.first == "phase") phase = parse_phase(kv.second);
        auto it = waf.defaults.find(phase);
        if (it != waf.defaults.end()) acts = merge_defaults(acts, it->second);
      }
      apply_actions(&rule, acts);
      if (is_child) {
        rule.phase = parent->phase;
        bool more = rule.has_chain;
        parent->children.push_back(rule);
        if (!more) parent = nullptr;
      } else {
        if (rule.id == 0) perr("rule id is required (line " + std::to_string(ln.first) + ")");
        if (id_count.count(rule.id)) perr("there is a another rule with id " + std::to_string(rule.id));
        id_count[rule.id]++;
        waf.rules.push_back(rule);
        if (rule.has_chain) parent = &waf.rules.back();
      }
    } else if (ignored_directive(d)) {
    } else {
      perr("unknown directive " + directive);
    }
  }
  if (parent) perr("unterminated chain");
  // The request path evaluates phases 1 and 2 (and phase-0 SecMarker records,
  // RuleGroup.Eval's "Phase_ == 0 always runs").  Rules of phases 3-5 are
  // parsed and validated like NewWAF does, then left out of the program: they
  // cannot change a phase 1-2 verdict (skip:N does not count rules of other
  // phases; their setvar / ctl run only after ProcessRequestBody).
  for (const IrRule& r : waf.rules) {
    if (r.phase != 1 && r.phase != 2) continue;
    if (!r.deferred.empty()) unsup(r.deferred + " (rule " + std::to_string(r.id) + ", phase " + std::to_string(r.phase) + ")");
    for (const IrRule& c : r.children)
      if (!c.deferred.empty()) unsup(c.deferred + " (chain of rule " + std::to_string(r.id) + ")");
  }
  waf.rules.erase(std::remove_if(waf.rules.begin(), waf.rules.end(), [](const IrRule& r) { return r.phase >= 3; }),
                  waf.rules.end());
  // SecMarkers no remaining skipAfter names (the response files' END-* markers)
  // are no-ops of every walk -- unless a skip:N counts them
  bool any_skip = false;
  std::set<std::string> targets;
  for (const IrRule& r : waf.rules) {
    any_skip = any_skip || r.skip > 0;
    if (!r.skip_after.empty()) targets.insert(r.skip_after);
  }
  if (!any_skip)
    waf.rules.erase(std::remove_if(waf.rules.begin(), waf.rules.end(),
                                   [&](const IrRule& r) { return !r.secmark.empty() && !targets.count(r.secmark); }),
                    waf.rules.end());
  return waf;
}

// ------------------------------------------------------------- lowering
struct Lower {
  Program* P;
  std::map<std::string, int> slots;
  std::map<std::string, int> markers;
  std::map<std::string, int> rm_groups;  // ctl removal groups: "t:<tag>" / "m:<msg>" -> bit
  std::map<std::string, int> dfa_cache;  // -1: no DFA (state cap), see nfa_cache
  std::map<std::string, int> nfa_cache;
  std::vector<std::pair<uint32_t, std::string>> tx_rx_vars;  // regex-keyed TX targets: (vars index, key regex)
  uint32_t cap;

  uint32_t str(const std::string& s) {
    uint32_t off = (uint32_t)P->strpool.size();
    P->strpool.insert(P->strpool.end(), s.begin(), s.end());
    P->strpool.push_back(0);
    return off;
  }
  int slot(const std::string& key) {
    std::string k = lower(key);
    auto it = slots.find(k);
    if (it != slots.end()) return it->second;
    int id = (int)slots.size();
    slots[k] = id;
    P->slot_names.push_back(str(k));
    P->slot_names.push_back((uint32_t)k.size());
    return id;
  }
  int rm_group(const std::string& key) {
    auto it = rm_groups.find(key);
    if (it != rm_groups.end()) return it->second;
    if (rm_groups.size() >= GI_MAX_RM_GROUPS) unsup("more than 32 distinct ctl:ruleRemove*ByTag / ByMsg values");
    const int id = (int)rm_groups.size();
    rm_groups[key] = id;
    return id;
  }
  int marker(const std::string& name) {
    auto it = markers.find(name);
    if (it != markers.end()) return it->second;
    int id = (int)markers.size();
    markers[name] = id;
    return id;
  }
  int add_dfa(const Dfa& d) {
    DDfa h{};
    h.n_states = d.n_states;
    h.n_classes = d.n_classes;
    h.start = d.start;
    h.accept = d.accept;
    h.trans_off = (uint32_t)P->trans.size();
    P->trans.insert(P->trans.end(), d.trans.begin(), d.trans.end());
    h.endacc_off = (uint32_t)P->u8pool.size();
    P->u8pool.insert(P->u8pool.end(), d.end_accept.begin(), d.end_accept.end());
    h.amap_off = (uint32_t)P->u8pool.size();
    P->u8pool.insert(P->u8pool.end(), d.amap.begin(), d.amap.end());
    h.nr_off = (uint32_t)P->nranges.size();
    h.nr_cnt = (uint32_t)d.nranges.size() / 3;
    P->nranges.insert(P->nranges.end(), d.nranges.begin(), d.nranges.end());
    h.byte_mode = d.byte_mode ? 1 : 0;
    h.multi = d.multi ? 1 : 0;
    if (d.multi) {
      h.combo_off = (uint32_t)P->u8pool.size();
      P->u8pool.insert(P->u8pool.end(), d.cls_combo.begin(), d.cls_combo.end());
      h.acc_off = (uint32_t)P->u64pool.size();
      P->u64pool.insert(P->u64pool.end(), d.acc.begin(), d.acc.end());
    }
    if (!d.byte_mode && h.nr_cnt > 0) {
      uint32_t c0 = d.nranges[2];
      bool uni = true;
      for (uint32_t k = 0; k < h.nr_cnt; k++)
        if (d.nranges[k * 3 + 2] != c0) uni = false;
      // ranges must cover every rune >= 0x80 (they do: the partition is total)
      h.nonascii_uniform = uni ? 1 : 0;
      h.nonascii_cls = (uint8_t)c0;
    }
    P->dfas.push_back(h);
    return (int)P->dfas.size() - 1;
  }
  // The sticky search DFA of `pattern`.  When it exceeds the state cap and
  // `nfa` is given (an @rx operator), the exact matcher is the pattern's NFA
  // tables instead (*nfa = DNfa index, returns -1); key / exception regexes
  // have no such fallback.
  int regex_dfa(const std::string& pattern, int32_t* nfa = nullptr) {
    std::string key = "rx:" + pattern;
    auto it = dfa_cache.find(key);
    if (it != dfa_cache.end()) {
      if (it->second < 0 && nfa) *nfa = nfa_cache[key];
      return it->second;
    }
    Regex re;
    std::string err;
    if (!re_parse(pattern, &re, &err)) perr("invalid regex " + pattern + ": " + err);
    Dfa d;
    if (!build_regex_dfa(re, &d, &err, cap)) {
      if (!nfa) unsup("regex " + pattern + ": " + err);
      NfaTables t;
      std::string nerr;
      if (!build_nfa_tables(re, &t, &nerr)) unsup("regex " + pattern + ": " + err + "; " + nerr);
      *nfa = add_nfa(t);
      nfa_cache[key] = *nfa;
      dfa_cache[key] = -1;
      return -1;
    }
    int id = add_dfa(d);
    dfa_cache[key] = id;
    return id;
  }
  int add_nfa(const NfaTables& t) {
    DNfa h{};
    h.n_classes = t.n_classes;
    h.n_pos = t.n_pos;
    h.words = t.words;
    h.amap_off = (uint32_t)P->u8pool.size();
    P->u8pool.insert(P->u8pool.end(), t.amap.begin(), t.amap.end());
    h.combo_off = (uint32_t)P->u8pool.size();
    P->u8pool.insert(P->u8pool.end(), t.cls_combo.begin(), t.cls_combo.end());
    h.nr_off = (uint32_t)P->nranges.size();
    h.nr_cnt = (uint32_t)t.nranges.size() / 3;
    P->nranges.insert(P->nranges.end(), t.nranges.begin(), t.nranges.end());
    h.cm_off = P->u64pool.size();
    P->u64pool.insert(P->u64pool.end(), t.cm.begin(), t.cm.end());
    h.follow_off = P->u64pool.size();
    P->u64pool.insert(P->u64pool.end(), t.follow.begin(), t.follow.end());
    P->nfas.push_back(h);
    return (int)P->nfas.size() - 1;
  }
  // Large phrase sets split into groups whose Aho-Corasick automata stay
  // below the state cap (a trie has at most 1 + total phrase bytes nodes).
  static constexpr size_t kPhraseGroupBytes = 40000;
  static std::vector<std::vector<std::string>> phrase_groups(const std::vector<std::string>& phrases) {
    std::vector<std::vector<std::string>> g(1);
    size_t bytes = 0;
    for (auto& p : phrases) {
      if (bytes + p.size() > kPhraseGroupBytes && !g.back().empty()) {
        g.emplace_back();
        bytes = 0;
      }
      g.back().push_back(p);
      bytes += p.size();
    }
    return g;
  }
  // the phrase automata of an operator: first DFA id, *ngroups = 0 (one
  // automaton) or the number of consecutive group automata
  int phrase_dfas(const std::vector<std::string>& phrases, bool fold, const std::string& key, uint32_t* ngroups) {
    size_t total = 0;
    for (auto& p : phrases) total += p.size();
    *ngroups = 0;
    if (total <= kPhraseGroupBytes) return phrase_dfa(phrases, fold, key);
    std::vector<Dfa> ds = phrase_group_dfas(phrases, fold);
    int first = -1;
    for (auto& d : ds) {
      const int id = add_dfa(d);
      if (first < 0) first = id;
    }
    *ngroups = (uint32_t)ds.size();
    return first;
  }
  // The group automata of a large phrase set, built on all host cores (each
  // group is an independent Aho-Corasick automaton) and kept for the phase-A
  // plan, which scans the same groups.
  std::map<std::pair<bool, std::vector<std::string>>, std::vector<Dfa>> group_cache;
  std::vector<Dfa> phrase_group_dfas(const std::vector<std::string>& phrases, bool fold) {
    auto key = std::make_pair(fold, phrases);
    auto it = group_cache.find(key);
    if (it != group_cache.end()) return it->second;
    const auto groups = phrase_groups(phrases);
    std::vector<Dfa> ds(groups.size());
    std::vector<std::string> errs(groups.size());
    std::vector<char> ok(groups.size(), 0);
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t k; (k = next.fetch_add(1)) < groups.size();)
        ok[k] = build_phrase_dfa(groups[k], fold, &ds[k], &errs[k], cap) ? 1 : 0;
    };
    const unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16));
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt && t < groups.size(); t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    for (size_t k = 0; k < groups.size(); k++)
      if (!ok[k]) unsup(errs[k]);
    group_cache[key] = ds;
    return ds;
  }
  int phrase_dfa(const std::vector<std::string>& phrases, bool fold, const std::string& key) {
    auto it = dfa_cache.find(key);
    if (it != dfa_cache.end()) return it->second;
    Dfa d;
    std::string err;
    if (!build_phrase_dfa(phrases, fold, &d, &err, cap)) unsup(err);
    int id = add_dfa(d);
    dfa_cache[key] = id;
    return id;
  }

  // %{...} macro template [upstream internal/macro]
  int tmpl(const std::string& s) {
    DTmpl t;
    t.part_begin = (uint32_t)P->tparts.size();
    size_t pos = 0;
    auto lit = [&](const std::string& l) {
      if (l.empty()) return;
      DTmplPart p{};
      p.kind = TP_LIT;
      p.off = str(l);
      p.len = (uint32_t)l.size();
      P->tparts.push_back(p);
    };
    for (;;) {
      size_t a = s.find("%{", pos);
      size_t b = a == std::string::npos ? a : s.find('}', a);
      if (a == std::string::npos || b == std::string::npos) {
        lit(s.substr(pos));
        break;
      }
      lit(s.substr(pos, a - pos));
      std::string ref = s.substr(a + 2, b - a - 2);
      size_t dot = ref.find('.');
      std::string name = upper(dot == std::string::npos ? ref : ref.substr(0, dot));
      std::string key = lower(dot == std::string::npos ? "" : ref.substr(dot + 1));
      DTmplPart p{};
      if (name == "TX") {
        p.kind = TP_TX;
        p.slot = slot(key);
      } else if (single_id(name) >= 0) {
        p.kind = TP_SINGLE;
        p.single = (uint8_t)single_id(name);
      } else if (name == "REQUEST_HEADERS") {
        p.kind = TP_HEADER;
        p.off = str(key);
        p.len = (uint32_t)key.size();
      } else if (name == "MATCHED_VAR" && key.empty()) {
        p.kind = TP_MV;
        P->mv_used = 1;
      } else if (name == "MATCHED_VAR_NAME" && key.empty()) {
        p.kind = TP_MVNAME;
        P->mv_used = 1;
      } else {
        unsup("unsupported macro %{" + ref + "}");
      }
      P->tparts.push_back(p);
      pos = b + 1;
    }
    t.part_count = (uint32_t)P->tparts.size() - t.part_begin;
    P->tmpls.push_back(t);
    return (int)P->tmpls.size() - 1;
  }
  bool tmpl_is_lit(int id, std::string* lit) {
    const DTmpl& t = P->tmpls[id];
    lit->clear();
    for (uint32_t k = 0; k < t.part_count; k++) {
      const DTmplPart& p = P->tparts[t.part_begin + k];
      if (p.kind != TP_LIT) return false;
      lit->append((const char*)&P->strpool[p.off], p.len);
    }
    return true;
  }

  int op(const IrRule& r) {
    DOp o{};
    o.negate = r.op_neg ? 1 : 0;
    o.dfa = -1;
    o.nfa = -1;
    o.tmpl = -1;
    o.pike = -1;
    const std::string& n = r.op_name;
    const std::string& a = r.op_arg;
    if (n == "ipmatch") {
      o.kind = OP_IPMATCH;
      size_t cnt = 0;
      const std::string recs = ipmatch_records(a, &cnt);
      o.arg_is_lit = 1;
      o.lit_off = str(recs);
      o.lit_len = (uint32_t)recs.size();
    } else if (n == "rx") {
      o.kind = OP_RX;
      o.dfa = regex_dfa("(?sm)" + a, &o.nfa);
    } else if (n == "pm") {
      o.kind = OP_PM;
      std::vector<std::string> phrases;
      std::string la = lower(a);
      size_t pos = 0;
      while (pos <= la.size()) {
        size_t sp = la.find(' ', pos);
        if (sp == std::string::npos) sp = la.size();
        if (sp > pos) phrases.push_back(la.substr(pos, sp - pos));
        pos = sp + 1;
      }
      o.dfa = phrase_dfas(phrases, true, "pm:" + la, &o.ngroups);
    } else if (n == "pmfromfile") {
      o.kind = OP_PM;
      std::string key = "pmf:";
      for (auto& p : r.phrases) key.append(p).push_back('\n');
      o.dfa = phrase_dfas(r.phrases, true, key, &o.ngroups);
    } else if (n == "detectsqli") {
      o.kind = OP_DETECT_SQLI;  // [upstream] detect_sqli.go (libinjection-go v0.2.2 IsSQLi; csrc/libinj.h)
    } else if (n == "detectxss") {
      o.kind = OP_DETECT_XSS;   // detect_xss.go (IsXSS)
    } else if (n == "unconditionalmatch") {
      o.kind = OP_UNCONDITIONAL;
    } else if (n == "nomatch") {
      o.kind = OP_NOMATCH;
    } else if (n == "validateurlencoding") {
      o.kind = OP_VALIDATE_URL_ENCODING;
    } else if (n == "validateutf8encoding") {
      o.kind = OP_VALIDATE_UTF8;
    } else if (n == "validatebyterange") {
      o.kind = OP_VALIDATE_BYTE_RANGE;
      std::stringstream ss(a);
      std::string part;
      while (std::getline(ss, part, ',')) {
        part = trim(part);
        if (part.empty()) continue;
        int64_t lo, hi;
        size_t dash = part.find('-');
        if (dash != std::string::npos) {
          if (!go_atoi(trim(part.substr(0, dash)), &lo) || !go_atoi(trim(part.substr(dash + 1)), &hi) ||
              lo < 0 || hi > 255 || lo > hi)
            perr("invalid byte range " + part);
        } else {
          if (!go_atoi(part, &lo) || lo < 0 || lo > 255) perr("invalid byte " + part);
          hi = lo;
        }
        for (int64_t x = lo; x <= hi; x++) o.bits[x >> 5] |= 1u << (x & 31);
      }
    } else {
      static const std::map<std::string, uint8_t> m = {
          {"contains", OP_CONTAINS}, {"containsword", OP_CONTAINSWORD}, {"streq", OP_STREQ},
          {"ipmatch", OP_IPMATCH},
          {"beginswith", OP_BEGINSWITH}, {"endswith", OP_ENDSWITH}, {"within", OP_WITHIN},
          {"eq", OP_EQ}, {"ge", OP_GE}, {"gt", OP_GT}, {"le", OP_LE}, {"lt", OP_LT}};
      o.kind = m.at(n);
      o.tmpl = tmpl(a);
      std::string lit;
      if (tmpl_is_lit(o.tmpl, &lit)) {
        o.arg_is_lit = 1;
        o.lit_off = str(lit);
        o.lit_len = (uint32_t)lit.size();
        int64_t v = 0;
        if (!go_atoi(lit, &v)) v = 0;
        o.has_num = 1;
        o.num = v;
        if (o.kind == OP_CONTAINS) o.dfa = phrase_dfa({lit}, false, "contains:" + lit);
        if (o.kind == OP_WITHIN) o.dfa = within_dfa(P->dfas, P->trans, P->u8pool, lit);
      }
    }
    P->ops.push_back(o);
    return (int)P->ops.size() - 1;
  }

  void vars(const IrRule& r, DRule* d) {
    d->var_begin = (uint32_t)P->vars.size();
    for (auto& v : r.vars) {
      if (known_unsupported_var(v.name)) unsup("unsupported variable " + v.name);
      DVarRef vr{};
      vr.count = v.count ? 1 : 0;
      vr.key_dfa = -1;
      vr.slot = -1;
      int sid = single_id(v.name);
      if (sid >= 0) {
        vr.var = (uint8_t)sid;
      } else {
        vr.var = (uint8_t)collection_ids().at(v.name);
        if (vr.var >= V_MATCHED_VAR) P->mv_used = 1;
        vr.ci = (vr.var == V_REQUEST_HEADERS || vr.var == V_REQUEST_HEADERS_NAMES || vr.var == V_TX ||
                 vr.var == V_MATCHED_VARS || vr.var == V_MATCHED_VARS_NAMES || vr.var == V_FILES ||
                 vr.var == V_FILES_NAMES || vr.var == V_FILES_SIZES || vr.var == V_FILES_TMPNAMES ||
                 vr.var == V_MULTIPART_PART_HEADERS) ? 1 : 0;  // coraza collections.NewMap
        if (v.key_rx) {
          vr.key_mode = 2;
          vr.key_dfa = regex_dfa(v.key);
          if (vr.var == V_TX) {
            tx_rx_vars.emplace_back((uint32_t)P->vars.size(), v.key);
            // "^literal": keys created at run time are tested by a prefix compare
            bool lit = v.key.size() >= 2 && v.key.size() <= 256 && v.key[0] == '^';
            for (size_t q = 1; lit && q < v.key.size(); q++) lit = !strchr("\\.+*?()[]{}|$^", v.key[q]);
            if (lit) {
              vr.slot = (int32_t)str(v.key.substr(1));
              vr.pre_len = (uint8_t)(v.key.size() - 1);
            }
          }
        } else if (!v.key.empty()) {
          vr.key_mode = 1;
          std::string k = vr.ci ? lower(v.key) : v.key;
          vr.key_off = str(k);
          vr.key_len = (uint32_t)k.size();
          if (vr.var == V_TX) vr.slot = slot(k);
        }
      }
      vr.exc_begin = (uint32_t)P->excs.size();
      for (auto& e : v.exc) {
        DExc x{};
        x.dfa = -1;
        if (e.second) {
          x.dfa = regex_dfa(e.first);
        } else {
          x.off = str(e.first);
          x.len = (uint32_t)e.first.size();
          x.hash = gi_fnv1a((const uint8_t*)e.first.data(), x.len, true);
        }
        P->excs.push_back(x);
      }
      vr.exc_count = (uint32_t)P->excs.size() - vr.exc_begin;
      P->vars.push_back(vr);
    }
    d->var_count = (uint32_t)P->vars.size() - d->var_begin;
  }

  // setvar fast forms (DAction.a = SV_*, .b operand); anything else stays
  // SV_GENERIC and runs the macro-expanding path (run_setvar).
  void classify_setvar(DAction* a) {
    const DTmpl& tm = P->tmpls[a->tmpl];
    auto lit_of = [&](const DTmplPart& p) {
      return std::string((const char*)&P->strpool[p.off], p.len);
    };
    a->a = SV_GENERIC;
    if (tm.part_count == 1 && P->tparts[tm.part_begin].kind == TP_LIT) {
      const std::string l = lit_of(P->tparts[tm.part_begin]);
      int64_t v;
      if (l.empty()) return;
      if (l[0] == '+' || l[0] == '-') {
        if (go_atoi(l.substr(1), &v)) {
          a->a = l[0] == '+' ? SV_ADD_CONST : SV_SUB_CONST;
          a->b = v;
        }
      } else if (go_atoi(l, &v) && std::to_string(v) == l) {
        a->a = SV_SET_INT;
        a->b = v;
      }
      return;
    }
    if (tm.part_count == 2 && P->tparts[tm.part_begin].kind == TP_LIT && P->tparts[tm.part_begin + 1].kind == TP_TX &&
        P->tparts[tm.part_begin + 1].slot >= 0) {
      const std::string l = lit_of(P->tparts[tm.part_begin]);
      if (l == "+" || l == "-") {
        a->a = l == "+" ? SV_ADD_SLOT : SV_SUB_SLOT;
        a->b = P->tparts[tm.part_begin + 1].slot;
      }
    }
  }

  // setvar whose key has a macro [upstream internal/actions/setvar.go: the key
  // is expanded per execution, then lowercased]: a run-time TX key (k_eval
  // dyn_slot).  Records how many executions / bytes the action can need per
  // request (DDynSite, gi_program.h) so the host sizes the dynamic TX area
  // exactly instead of guessing.
  void dyn_setvar(const IrRule& r, const IrNd& nd) {
    DAction a{};
    a.kind = nd.sv_remove ? A_SETVAR_DEL : A_SETVAR;
    a.slot = -1;
    a.aux = tmpl(nd.sv_key);
    a.tmpl = nd.sv_remove ? -1 : tmpl(nd.sv_value);
    if (a.kind == A_SETVAR) classify_setvar(&a);
    DDynSite ds{};
    ds.mm = r.multimatch ? (uint32_t)r.transforms.size() + 1 : 1;
    // the link's transformation chain: growth of the matched value on ASCII / any input
    uint32_t ga = 1, gn = 1;
    bool ascii = true;
    for (const std::string& tn : r.transforms) {
      uint8_t code = 0;
      transform_code(tn, &code);
      switch (code) {
        case T_LOWERCASE:
        case T_UTF8TOUNICODE:  // a non-ASCII byte: U+FFFD (3 B) / "%uXXXX" for a 2-byte rune
          ga *= ascii ? 1 : 3;
          gn *= 3;
          break;
        case T_URLENCODE: ga *= 3; gn *= 3; break;
        case T_HEXENCODE: ga *= 2; gn *= 2; break;
        case T_BASE64ENCODE: ga *= 2; gn *= 2; break;
        case T_SHA1: case T_MD5: case T_LENGTH: ds.fixed += 64; break;
        case T_URLDECODE: case T_URLDECODEUNI: case T_HTMLENTITYDECODE: case T_JSDECODE: case T_CSSDECODE:
        case T_BASE64DECODE: case T_BASE64DECODEEXT: case T_HEXDECODE: case T_ESCAPESEQDECODE:
          ascii = false;  // can emit non-ASCII bytes from ASCII input
          break;
        default: break;
      }
      if (gn > 729) unsup("setvar with a macro key after a transformation chain that grows values " +
                          std::to_string(gn) + "x");
    }
    ds.g_ascii = ga;
    ds.g_any = gn;
    const bool own_capture = r.capture && r.has_op && r.op_name == "rx" && !r.op_neg;
    auto parts = [&](int tid) {
      if (tid < 0) return;
      const DTmpl& tm = P->tmpls[tid];
      for (uint32_t k = 0; k < tm.part_count; k++) {
        const DTmplPart& p = P->tparts[tm.part_begin + k];
        if (p.kind == TP_LIT) {
          ds.lit += p.len;
        } else if (p.kind == TP_MV) {
          ds.n_val++;
        } else if (p.kind == TP_MVNAME) {
          ds.n_mvname++;
        } else if (p.kind == TP_TX && own_capture) {
          const uint32_t no = P->slot_names[2 * p.slot], nn = P->slot_names[2 * p.slot + 1];
          const bool digit = nn == 1 && P->strpool[no] >= '0' && P->strpool[no] <= '8';
          if (digit) ds.n_val++;
          else ds.n_big++;
        } else {
          ds.n_big++;
        }
      }
    };
    parts(a.aux);
    parts(a.tmpl);
    for (const IrVar& v : r.vars) {
      const int sid = single_id(v.name);
      if (sid >= 0 || v.count) ds.nsingles++;
      else if (v.name == "REQUEST_HEADERS_NAMES") ds.hdr_names++;
      else if (v.name == "REQUEST_HEADERS") ds.hdr_vals++;
      else if (v.name == "TX" || v.name.rfind("MATCHED_VAR", 0) == 0)
        unsup("setvar with a macro key on a rule reading " + v.name);
      else ds.other_coll++;
    }
    ds.no_targets = r.vars.empty() ? 1 : 0;
    {  // the key's leading literal (which static TX names the key could ever produce)
      const DTmpl& tm = P->tmpls[a.aux];
      const DTmplPart& p0 = P->tparts[tm.part_begin];
      std::string pre = tm.part_count && p0.kind == TP_LIT ? lower(std::string((const char*)&P->strpool[p0.off], p0.len)) : "";
      ds.prefix_off = str(pre);
      ds.prefix_len = (uint32_t)pre.size();
    }
    P->dyn_sites.push_back(ds);
    P->acts.push_back(a);
  }

  void actions(const IrRule& r, DRule* d) {
    d->act_begin = (uint32_t)P->acts.size();
    for (auto& nd : r.nd) {
      if (nd.is_setvar) {
        if (nd.sv_key.find("%{") != std::string::npos) {
          dyn_setvar(r, nd);
          continue;
        }
        DAction a{};
        a.kind = nd.sv_remove ? A_SETVAR_DEL : A_SETVAR;
        a.slot = slot(nd.sv_key);
        a.tmpl = nd.sv_remove ? -1 : tmpl(nd.sv_value);
        if (a.kind == A_SETVAR) classify_setvar(&a);
        P->acts.push_back(a);
      } else if (nd.ctl_name == "ruleremovebyid") {
        std::stringstream ss(nd.ctl_value);
        std::string part;
        while (std::getline(ss, part, ' ')) {
          part = trim(part);
          if (part.empty()) continue;
          DAction a{};
          a.kind = A_CTL_RULE_REMOVE_ID;
          int64_t lo, hi;
          size_t dash = part.find('-');
          if (dash != std::string::npos) {
            if (!go_atoi(part.substr(0, dash), &lo) || !go_atoi(part.substr(dash + 1), &hi))
              perr("invalid ctl:ruleRemoveById " + part);
          } else {
            if (!go_atoi(part, &lo)) perr("invalid ctl:ruleRemoveById " + part);
            hi = lo;
          }
          a.a = lo;
          a.b = hi;
          P->acts.push_back(a);
        }
      } else if (nd.ctl_name == "ruleremovebytag" || nd.ctl_name == "ruleremovebymsg") {
        // [upstream internal/actions/ctl.go]: every rule whose tags contain the
        // value (whose msg equals it) is removed by id for the transaction
        DAction a{};
        a.kind = A_CTL_RULE_REMOVE_GROUP;
        a.a = rm_group((nd.ctl_name == "ruleremovebytag" ? "t:" : "m:") + nd.ctl_value);
        P->acts.push_back(a);
      } else if (nd.ctl_name == "ruleremovetargetbyid" || nd.ctl_name == "ruleremovetargetbytag" ||
                 nd.ctl_name == "ruleremovetargetbymsg") {
        // "ID[-ID];VARIABLE[:key]" / "TAG;VARIABLE[:key]" / "MSG;VARIABLE[:key]" [upstream internal/actions/ctl.go]
        const size_t semi = nd.ctl_value.find(';');
        if (semi == std::string::npos) perr("invalid ctl:" + nd.ctl_name + " " + nd.ctl_value);
        const std::string ids = trim(nd.ctl_value.substr(0, semi)), tgt = trim(nd.ctl_value.substr(semi + 1));
        int64_t lo, hi;
        if (nd.ctl_name != "ruleremovetargetbyid") {
          lo = GI_RM_GROUP_MODE;
          hi = rm_group((nd.ctl_name == "ruleremovetargetbytag" ? "t:" : "m:") + ids);
        } else if (!parse_id_range(ids, &lo, &hi)) {
          perr("invalid ctl:ruleRemoveTargetById " + nd.ctl_value);
        }
        const size_t colon = tgt.find(':');
        const std::string vname = upper(trim(tgt.substr(0, colon)));
        const std::string key = colon == std::string::npos ? "" : lower(tgt.substr(colon + 1));
        int vid = single_id(vname);
        if (vid < 0) {
          auto it = collection_ids().find(vname);
          if (it == collection_ids().end()) unsup("ctl:ruleRemoveTargetById variable " + vname);
          vid = it->second;
        }
        DAction a{};
        a.kind = A_CTL_RULE_REMOVE_TARGET;
        a.a = lo;
        a.b = hi;
        a.slot = vid;
        a.tmpl = (int32_t)str(key);
        a.aux = (int32_t)key.size();
        P->acts.push_back(a);
      } else if (nd.ctl_name == "ruleengine") {
        DAction a{};
        a.kind = A_CTL_RULE_ENGINE;
        std::string v = lower(nd.ctl_value);
        a.a = v == "on" ? ENGINE_ON : v == "off" ? ENGINE_OFF : v == "detectiononly" ? ENGINE_DETECTION_ONLY : -1;
        if (a.a < 0) perr("invalid ctl:ruleEngine " + nd.ctl_value);
        P->acts.push_back(a);
      } else if (nd.ctl_name == "requestbodyprocessor") {
        DAction a{};
        a.kind = A_CTL_BODY_PROCESSOR;
        std::string v = upper(nd.ctl_value);
        a.a = v == "URLENCODED" ? BP_URLENCODED : v == "JSON" ? BP_JSON : v == "XML" ? BP_XML
              : v == "MULTIPART" ? BP_MULTIPART : -1;
        if (a.a < 0) perr("invalid ctl:requestBodyProcessor " + nd.ctl_value);
        P->acts.push_back(a);
      } else if (nd.ctl_name == "requestbodyaccess") {
        DAction a{};
        a.kind = A_CTL_BODY_ACCESS;
        a.a = lower(nd.ctl_value) == "on" ? 1 : 0;
        P->acts.push_back(a);
      }
      else if (nd.ctl_name == "forcerequestbodyvariable") {
        DAction a{};
        a.kind = A_CTL_FORCE_BODY;
        std::string v = lower(nd.ctl_value);
        a.a = (v == "on" || v == "true" || v == "1") ? 1 : 0;
        P->acts.push_back(a);
      }
    }
    d->act_count = (uint32_t)P->acts.size() - d->act_begin;
  }

  // ---------------------------------------------------- phase-A scan plan
  struct PatEntry {
    uint32_t slot;
    bool negate;
    int kind;  // 0 regex, 1 phrases (fold), 2 literal (case-sensitive)
    std::string rx;
    std::vector<std::string> phrases;
    uint64_t fmask;  // admitting filters (global filter ids)
  };
  std::map<std::string, uint32_t> gfilter_ids;  // global (deduplicated) filters: key -> id
  struct StreamBuild {
    DStream s;
    std::vector<DFilter> filters;
    std::vector<uint8_t> gids;  // global filter id of each stream filter
    std::vector<std::string> fkeys;
    std::vector<PatEntry> pats;
    std::vector<DScanVal> vals;
  };
  std::vector<StreamBuild> sbuild;
  std::vector<uint32_t> relaxed_slots;  // hit slots whose phase-A automaton is a superset relaxation
  uint32_t n_det = 0;  // streams with detect vals (DStream.det_id)
  std::map<std::string, size_t> sindex;

  // body collections phase A does not scan (part headers, XML): tested by k_eval on a clear bit.
  // FILES / FILES_NAMES / FILES_SIZES come out of k_mpparse's speculative
  // multipart parse before phase A and are scanned like ARGS_POST.
  static bool residual_collection(const std::string& n) {
    return n == "FILES_TMPNAMES" || n == "MULTIPART_PART_HEADERS" || n == "XML";
  }
  static bool immutable_single(int sid) {
    return sid == S_REQUEST_METHOD || sid == S_REQUEST_PROTOCOL || sid == S_REQUEST_URI ||
           sid == S_REQUEST_URI_RAW || sid == S_REQUEST_LINE || sid == S_REQUEST_FILENAME ||
           sid == S_REQUEST_BASENAME || sid == S_QUERY_STRING || sid == S_REMOTE_ADDR || sid == S_REMOTE_PORT ||
           sid == S_SERVER_NAME;
  }

  // Does the link's transformation chain + operator reject the empty value?
  // (Every transformation here maps "" to ""; the operator finds nothing in "".)
  static bool link_rejects_empty(const IrRule& r) {
    if (!r.has_op || r.op_neg || r.multimatch) return false;
    for (const auto& tf : r.transforms) {
      const std::string t = lower(tf);
      if (t == "length" || t == "sha1" || t == "md5") return false;
    }
    const std::string& n = r.op_name;
    if (n == "rx") {
      Regex re;
      Dfa d;
      std::string err;
      if (!re_parse("(?sm)" + r.op_arg, &re, &err) || !build_regex_dfa(re, &d, &err)) return false;
      return !dfa_host_match(d, (const uint8_t*)"", 0);
    }
    if (n == "pm" || n == "pmfromfile") return !r.phrases.empty() || !trim(r.op_arg).empty();
    if (n == "contains" || n == "containsword") return !r.op_arg.empty() && r.op_arg.find("%{") == std::string::npos;
    return n == "detectsqli" || n == "detectxss" || n == "validatebyterange" || n == "validateurlencoding" ||
           n == "validateutf8encoding";
  }

  // Assigns a hit slot and registers the link's patterns, or returns -1 when
  // the link stays interpreter-only (TX / count targets, macro arguments,
  // operators without an automaton form, mutable singles).
  bool no_scan = false;  // the current top-level rule sits behind a paranoia gate (gated_rules)
  // capture analysis (capture_analysis): every capture is observable, or only these links'
  bool cap_global = true;
  std::set<const IrRule*> cap_links;
  std::map<const IrRule*, std::string> pa_rx;  // first link -> its phase-A pattern (within_chain_filters)

  int32_t plan(const IrRule& r, const DRule& d, uint8_t* flags, uint8_t* flags2) {
    if (!r.has_op || no_scan) return -1;
    const std::string& n = r.op_name;
    // A link whose targets are all collection counts (&ARGS_POST:_charset_) and
    // whose numeric comparison fails on a zero count ("!@eq 0"): phase A sets its
    // bit iff some entry the targets admit exists (an always-true value test on
    // their filters), so a clear bit means every count is 0 and the link cannot
    // match -- the interpreter no longer walks a 2 500-field ARGS_POST for it.
    bool count_exists = false;
    {
      bool any = false, all = true;
      for (auto& v : r.vars) {
        any = any || v.count;
        all = all && v.count;
      }
      if (any) {
        if (!all || r.multimatch) return -1;
        const bool cmp = n == "eq" || n == "ge" || n == "gt" || n == "le" || n == "lt";
        int64_t k = 0;
        if (!cmp || r.op_arg.find("%{") != std::string::npos || !go_atoi(trim(r.op_arg), &k)) return -1;
        bool m0 = n == "eq" ? 0 == k : n == "ge" ? 0 >= k : n == "gt" ? 0 > k : n == "le" ? 0 <= k : 0 < k;
        if (r.op_neg) m0 = !m0;
        if (m0) return -1;  // a zero count matches: the bit could not settle it
        for (auto& v : r.vars)
          if (single_id(v.name) >= 0 || v.name == "TX" || v.name.rfind("MATCHED_VAR", 0) == 0 ||
              residual_collection(v.name))
            return -1;
        count_exists = true;
      }
    }
    bool scannable = n == "rx" || n == "pm" || n == "pmfromfile" || n == "validatebyterange" || n == "validateurlencoding" ||
                     n == "validateutf8encoding" || n == "detectsqli" || n == "detectxss" ||
                     (n == "contains" && r.op_arg.find("%{") == std::string::npos) || count_exists;
    if (!scannable) return -1;
    bool bodydep = false, residual = false, res_single = false, rb_only = true;
    for (auto& v : r.vars) {
      if (v.count && !count_exists) return -1;
      int sid = single_id(v.name);
      if (sid >= 0 && !immutable_single(sid)) residual = res_single = true;  // tested by k_eval on a clear bit
      if (sid >= 0 && !immutable_single(sid) && sid != S_REQUEST_BODY) rb_only = false;
      if (sid < 0 && v.name == "TX") return -1;
      if (v.name.rfind("MATCHED_VAR", 0) == 0) return -1;  // transaction state, not a request variable
      if (residual_collection(v.name)) residual = true;  // body collections phase A does not scan
      if (v.name == "ARGS" || v.name == "ARGS_POST" || v.name == "ARGS_NAMES" || v.name == "ARGS_POST_NAMES" ||
          v.name == "FILES" || v.name == "FILES_NAMES" || v.name == "FILES_SIZES")
        bodydep = true;
    }
    // multiMatch (rule.go executeTransformationsMultimatch) tests the value
    // after every prefix of the chain: its patterns go into one stream per
    // prefix, all on the link's slot (the bit ORs the candidates: exact
    // superset).  The residual clear-bit path and k_body test final values
    // only, so a multiMatch link with a residual single stays interpreter-only;
    // one whose residual targets are all body collections (XML, FILES*, part
    // headers) keeps its phase-A bit: k_eval treats any present residual value
    // as "maybe" and evaluates the whole link.
    if (r.multimatch && residual)
      for (auto& v : r.vars)
        if (single_id(v.name) >= 0 && !immutable_single(single_id(v.name))) return -1;
    // a detect link reading REQUEST_BODY would go to k_body, which does not run libinjection: interpreter-only
    if ((n == "detectsqli" || n == "detectxss") && residual)
      for (auto& v : r.vars)
        if (v.name == "REQUEST_BODY") return -1;
    const int32_t slot = (int32_t)P->n_hit_slots++;
    if (bodydep) *flags |= RF_BODYDEP;
    if (residual) *flags |= RF_RESIDUAL;
    if (residual && !res_single) *flags2 |= RF2_RESID_COLL;  // only body collections: empty without such a body
    if (residual && res_single && rb_only && link_rejects_empty(r)) *flags2 |= RF2_RESID_RB;
    const DOp& o = P->ops[d.op];
    DVarRef* vrs = &P->vars[d.var_begin];
    for (uint32_t vi = 0; vi < d.var_count; vi++) {
      DVarRef& vr = vrs[vi];
      if ((vr.var < S_COUNT && !immutable_single(vr.var)) || vr.var == V_FILES_TMPNAMES ||
          vr.var == V_MULTIPART_PART_HEADERS || vr.var == V_XML) {
        vr.residual = 1;
        continue;
      }
      DFilter f{};
      f.key_dfa = -1;
      f.single = GI_NO_SINGLE;
      if (vr.var < S_COUNT) {
        f.single = vr.var;
      } else {
        uint8_t mask = 0;
        bool names = false;
        switch (vr.var) {
          case V_ARGS_GET: mask = 1 << FK_ARG_GET; break;
          // ARG_POST items come from k_collect's speculative body parse
          case V_ARGS: mask = (1 << FK_ARG_GET) | (1 << FK_ARG_POST); break;
          case V_ARGS_POST: mask = 1 << FK_ARG_POST; break;
          case V_ARGS_POST_NAMES: mask = 1 << FK_ARG_POST; names = true; break;
          case V_REQUEST_HEADERS: mask = 1 << FK_HEADER; break;
          case V_REQUEST_COOKIES: mask = 1 << FK_COOKIE; break;
          case V_ARGS_GET_NAMES: mask = 1 << FK_ARG_GET; names = true; break;
          case V_ARGS_NAMES: mask = (1 << FK_ARG_GET) | (1 << FK_ARG_POST); names = true; break;
          case V_REQUEST_HEADERS_NAMES: mask = 1 << FK_HEADER; names = true; break;
          case V_REQUEST_COOKIES_NAMES: mask = 1 << FK_COOKIE; names = true; break;
          // multipart collections: k_mpparse's fields (key "" or the file name)
          case V_FILES: mask = 1 << FK_FILE; break;
          case V_FILES_NAMES: mask = 1 << FK_FILE_NAME; break;
          case V_FILES_SIZES: mask = 1 << FK_FILE_SIZE; break;
          default: break;  // XML, part headers, FILES_TMPNAMES: residual (above)
        }
        if (!mask) continue;
        f.kind_mask = mask;
        f.names = names;
        f.key_mode = vr.key_mode;
        f.ci = vr.ci;
        f.key_dfa = vr.key_dfa;
        f.key_off = vr.key_off;
        f.key_len = vr.key_len;
        if (vr.key_mode == 1) f.key_hash = gi_fnv1a(&P->strpool[vr.key_off], vr.key_len, false);
        f.exc_begin = vr.exc_begin;
        f.exc_count = vr.exc_count;
      }
      for (uint32_t plen = r.multimatch ? 0 : d.tchain_len; plen <= d.tchain_len; plen++) {
      const std::string skey((const char*)&P->tchains[d.tchain_off], plen);
      std::string fkey((const char*)&f, 5);
      if (f.key_mode == 1) fkey.append((const char*)&P->strpool[f.key_off], f.key_len);
      fkey.append("|" + std::to_string(f.key_dfa) + "|");
      for (uint32_t e = 0; e < f.exc_count; e++) {
        const DExc& x = P->excs[f.exc_begin + e];
        fkey.append(std::to_string(x.dfa) + ":");
        fkey.append((const char*)&P->strpool[x.off], x.len);
        fkey.push_back(',');
      }
      // find the stream part holding (or able to take) this filter
      size_t si = SIZE_MAX;
      uint32_t fid = 0;
      for (int part = 0; si == SIZE_MAX; part++) {
        std::string k = skey + "#" + std::to_string(part);
        auto it = sindex.find(k);
        if (it == sindex.end()) {
          StreamBuild sb;
          sb.s = DStream{};
          sb.s.tchain_off = d.tchain_off;
          sb.s.tchain_len = plen;
          sindex[k] = sbuild.size();
          sbuild.push_back(sb);
          it = sindex.find(k);
        }
        StreamBuild& sb = sbuild[it->second];
        auto fit = std::find(sb.fkeys.begin(), sb.fkeys.end(), fkey);
        if (fit != sb.fkeys.end()) {
          si = it->second;
          fid = (uint32_t)(fit - sb.fkeys.begin());
        } else if (sb.fkeys.size() < GI_MAX_FILTERS) {
          auto git = gfilter_ids.find(fkey);
          if (git == gfilter_ids.end()) {
            if (gfilter_ids.size() >= GI_MAX_GFILTERS) unsup("more than 64 distinct phase-A variable filters");
            git = gfilter_ids.emplace(fkey, (uint32_t)P->filters.size()).first;
            P->filters.push_back(f);
            if (f.single != GI_NO_SINGLE) {
              P->item_singles |= 1u << f.single;
            } else {
              for (int k = FK_ARG_GET; k <= FK_FILE_SIZE; k++)
                if ((f.kind_mask >> k) & 1) P->item_sides[k] |= f.names ? 2 : 1;
            }
          }
          sb.gids.push_back((uint8_t)git->second);
          sb.fkeys.push_back(fkey);
          sb.filters.push_back(f);
          sb.s.kind_mask |= f.kind_mask;
          si = it->second;
          fid = (uint32_t)sb.fkeys.size() - 1;
        }
      }
      StreamBuild& sb = sbuild[si];
      if (o.kind == OP_VALIDATE_BYTE_RANGE || o.kind == OP_VALIDATE_URL_ENCODING || o.kind == OP_VALIDATE_UTF8 ||
          o.kind == OP_DETECT_SQLI || o.kind == OP_DETECT_XSS || count_exists) {
        bool merged = false;
        for (auto& sv : sb.vals)
          if (sv.slot == (uint32_t)slot) sv.fmask |= 1ull << sb.gids[fid], merged = true;
        if (merged) continue;
        DScanVal sv{};
        sv.kind = count_exists ? (uint8_t)OP_UNCONDITIONAL : o.kind;
        sv.negate = count_exists ? 0 : o.negate;
        sv.fmask = 1ull << sb.gids[fid];
        sv.slot = (uint32_t)slot;
        for (int k = 0; k < 8; k++) sv.bits[k] = o.bits[k];
        sb.vals.push_back(sv);
        continue;
      }
      bool merged = false;
      for (auto& pe : sb.pats)
        if (pe.slot == (uint32_t)slot) pe.fmask |= 1ull << sb.gids[fid], merged = true;
      if (merged) continue;
      PatEntry pe;
      pe.slot = (uint32_t)slot;
      pe.negate = o.negate != 0;
      pe.fmask = 1ull << sb.gids[fid];
      if (o.kind == OP_RX) {
        pe.kind = 0;
        const auto ov = pa_rx.find(&r);
        pe.rx = ov != pa_rx.end() ? ov->second : "(?sm)" + r.op_arg;
      } else if (o.kind == OP_PM && r.op_name == "pmfromfile") {
        pe.kind = 1;
        pe.phrases = r.phrases;
      } else if (o.kind == OP_PM) {
        pe.kind = 1;
        std::string la = lower(r.op_arg);
        size_t pos = 0;
        while (pos <= la.size()) {
          size_t sp = la.find(' ', pos);
          if (sp == std::string::npos) sp = la.size();
          if (sp > pos) pe.phrases.push_back(la.substr(pos, sp - pos));
          pos = sp + 1;
        }
      } else {  // @contains literal
        pe.kind = 2;
        pe.phrases.push_back(r.op_arg);
      }
      sb.pats.push_back(pe);
      }  // prefix streams
    }
    return slot;
  }

  struct AutoBuild {
    Dfa d;
    std::vector<const PatEntry*> pes;
  };

  static uint32_t al16(uint32_t x) { return (x + 15) & ~15u; }
  // LDS footprint of one automaton in a job image (see DJob in gi_program.h)
  static uint32_t img_bytes(const Dfa& d) {
    uint32_t t = al16(d.n_states * d.n_classes * 2);
    uint32_t a = al16((uint32_t)d.amap.size());
    uint32_t c = d.multi ? al16((uint32_t)d.cls_combo.size()) : 0;
    uint32_t e = al16(d.n_states * (d.multi ? 8 : 1));
    return t + a + c + e;
  }
  // automaton fits an LDS image at all (u16 state ids with the union flag bit,
  // classes addressable through the joint u8-per-automaton class map)
  static bool img_ok(const Dfa& d) { return d.n_states < 0x8000 && d.n_classes <= 255; }
  static bool lds_ok(const Dfa& d, uint32_t nfilt) {
    return img_ok(d) && GI_JAMAP_BYTES + img_bytes(d) + al16(nfilt * 8) + al16(d.n_pat * 4) <= GI_BIG_LDS_BYTES;
  }
  void img_put(uint32_t img_off, const void* p, size_t n, int32_t* at) {
    *at = (int32_t)(P->images.size() - img_off);
    const uint8_t* b = (const uint8_t*)p;
    P->images.insert(P->images.end(), b, b + n);
    P->images.resize(img_off + al16((uint32_t)(P->images.size() - img_off)), 0);
  }

  void finish_streams() {
    const uint32_t kUnionTableBytes = 48 * 1024;  // LDS-resident union automata
    std::ostringstream js;
    js << "{\"streams\":[";
    bool first_s = true;
    // the gate's prefix links (RF2_PREFIX, marked before the plan): their
    // patterns get automata and jobs of their own, so the first stage can run
    // them over body fields without the other patterns of their streams
    std::vector<char> slot_prefix(P->n_hit_slots, 0);
    for (const DRule& d : P->rules)
      if (d.hit_slot >= 0 && (uint32_t)d.hit_slot < P->n_hit_slots && (d.flags2 & RF2_PREFIX)) slot_prefix[d.hit_slot] = 1;
    auto pe_prefix = [&](const PatEntry& pe) { return pe.slot < slot_prefix.size() && slot_prefix[pe.slot]; };
    for (auto& sb : sbuild) {
      std::stable_sort(sb.pats.begin(), sb.pats.end(), [&](const PatEntry& a, const PatEntry& b) {
        const bool pa = pe_prefix(a), pb = pe_prefix(b);
        return pa != pb ? pa : a.fmask < b.fmask;
      });
      // 1. automata: greedy union packing
      std::vector<AutoBuild> autos;
      std::vector<std::unique_ptr<Regex>> owned;
      std::vector<const Regex*> cur;
      std::vector<const PatEntry*> curp;
      Dfa curd;
      std::string err;
      auto flush = [&]() {
        if (cur.empty()) return;
        autos.push_back({std::move(curd), curp});
        cur.clear();
        curp.clear();
      };
      // A pattern's phase-A automaton: its exact DFA, or -- when that exceeds
      // the state cap -- the DFA of a superset relaxation (regex.h
      // relax_regex): a prefilter, since the hit bit only has to be a superset
      // (k_eval re-evaluates the link exactly, on the NFA tables).  A negated
      // operator has no superset filter: false (the link is always "maybe").
      auto single_or_relaxed = [&](const PatEntry& pe, const Regex& re, Dfa* out) -> bool {
        if (build_regex_dfa(re, out, &err, cap)) return true;
        if (pe.negate || pe.kind != 0) return false;
        for (int lvl = 1; lvl <= 3; lvl++) {
          Regex rr = re;
          relax_regex(&rr, lvl);
          if (build_regex_dfa(rr, out, &err, cap)) {
            relaxed_slots.push_back(pe.slot);
            return true;
          }
        }
        return false;
      };
      // Pass 1: the automata of patterns that never share a union (large
      // phrase sets, non-ASCII phrases, negated operators) -- kept per pattern
      // position -- and the list of patterns that may (packed in pass 2).
      std::vector<std::vector<AutoBuild>> fixed(sb.pats.size());
      std::vector<char> is_union(sb.pats.size(), 0);
      std::vector<std::pair<const PatEntry*, std::unique_ptr<Regex>>> unionable;
      for (size_t pi = 0; pi < sb.pats.size(); pi++) {
        const PatEntry& pe = sb.pats[pi];
        auto re = std::make_unique<Regex>();
        bool ok;
        size_t pbytes = 0;
        for (auto& p : pe.phrases) pbytes += p.size();
        if (pe.kind != 0 && pbytes > kPhraseGroupBytes) {  // a large phrase set: its group automata
          if (pe.negate) {  // "no group matches" is not a per-automaton bit: always "maybe"
            P->always_slots.push_back(pe.slot);
            continue;
          }
          for (auto& d : phrase_group_dfas(pe.phrases, pe.kind == 1)) fixed[pi].push_back({std::move(d), {&pe}});
          continue;
        }
        if (pe.kind == 0) {
          ok = re_parse(pe.rx, re.get(), &err);
          if (!ok) perr("invalid regex " + pe.rx + ": " + err);
        } else {
          ok = phrases_to_regex(pe.phrases, pe.kind == 1, re.get());
        }
        if (!ok) {  // non-ASCII phrase: its own byte-mode automaton
          Dfa d;
          if (!build_phrase_dfa(pe.phrases, pe.kind == 1, &d, &err, cap)) unsup(err);
          fixed[pi].push_back({std::move(d), {&pe}});
          continue;
        }
        if (pe.negate) {  // negated operators stay out of union automata (the scan emits union hits eagerly)
          Dfa single;
          if (!single_or_relaxed(pe, *re, &single)) {  // no automaton: the link is always "maybe"
            P->always_slots.push_back(pe.slot);
            continue;
          }
          fixed[pi].push_back({std::move(single), {&pe}});
          continue;
        }
        is_union[pi] = 1;
        unionable.emplace_back(&pe, std::move(re));
      }
      // Pass 2, greedy packing: each union automaton takes the next patterns
      // (<= 64) until adding one more would leave 16384 states or the LDS
      // table budget (a failing trial stops as soon as its states exceed the
      // byte budget: build_union_dfa's byte_budget).  A pattern that does not
      // fit even alone gets its own sticky DFA (or is always "maybe").  Runs of
      // kPackChunk patterns are packed independently, on all host cores (a
      // chunk boundary also ends a union: the plan does not depend on the
      // thread count).
      constexpr size_t kPackChunk = 512;
      size_t n_pre_u = 0;  // the prefix patterns lead the list: a union never mixes them with the others
      while (n_pre_u < unionable.size() && pe_prefix(*unionable[n_pre_u].first)) n_pre_u++;
      struct Group {
        AutoBuild ab;
        size_t n = 0;         // patterns of the group
        bool unioned = false;
        bool always = false;  // no automaton at all
        bool relaxed = false;  // the automaton is a superset relaxation of its one pattern
      };
      std::vector<std::pair<size_t, size_t>> chunks;  // [begin, end): kPackChunk runs of each part
      for (size_t b0 = 0; b0 < n_pre_u; b0 += kPackChunk) chunks.push_back({b0, std::min(n_pre_u, b0 + kPackChunk)});
      for (size_t b0 = n_pre_u; b0 < unionable.size(); b0 += kPackChunk)
        chunks.push_back({b0, std::min(unionable.size(), b0 + kPackChunk)});
      const size_t nchunks = chunks.size();
      std::vector<std::vector<Group>> packed(nchunks);
      auto pack_chunk = [&](size_t ch) {
        std::string lerr;
        std::vector<Group>& out = packed[ch];
        const size_t end = chunks[ch].second;
        for (size_t i = chunks[ch].first; i < end;) {
          const size_t maxn = std::min<size_t>(64, end - i);
          auto fits = [&](size_t n, Dfa* d) {
            std::vector<const Regex*> rs;
            for (size_t k = 0; k < n; k++) rs.push_back(unionable[i + k].second.get());
            return build_union_dfa(rs, d, &lerr, 16384, 4 * kUnionTableBytes) && img_bytes(*d) <= kUnionTableBytes;
          };
          size_t lo = 0;  // a union of the next lo patterns fits; lo + 1 does not
          Dfa best;
          while (lo < maxn) {
            Dfa t;
            if (!fits(lo + 1, &t)) break;
            lo++;
            best = std::move(t);
          }
          Group g;
          if (lo > 0) {
            for (size_t k = 0; k < lo; k++) g.ab.pes.push_back(unionable[i + k].first);
            g.ab.d = std::move(best);
            g.n = lo;
            g.unioned = true;
            out.push_back(std::move(g));
            i += lo;
            continue;
          }
          // too large for an LDS union automaton: single sticky DFA (global tables)
          const PatEntry& pe = *unionable[i].first;
          bool ok = build_regex_dfa(*unionable[i].second, &g.ab.d, &lerr, cap);
          for (int lvl = 1; !ok && !pe.negate && pe.kind == 0 && lvl <= 3; lvl++) {
            Regex rr = *unionable[i].second;
            relax_regex(&rr, lvl);
            ok = build_regex_dfa(rr, &g.ab.d, &lerr, cap);
            g.relaxed = ok;
          }
          g.ab.pes = {&pe};
          g.n = 1;
          g.always = !ok;  // no automaton: the link is always "maybe"
          out.push_back(std::move(g));
          i++;
        }
      };
      {
        std::atomic<size_t> next{0};
        auto work = [&]() {
          for (size_t ch; (ch = next.fetch_add(1)) < nchunks;) pack_chunk(ch);
        };
        const unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16));
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt && t < nchunks; t++) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
      }
      // Emit in pattern order as a one-pattern-at-a-time greedy pass would: a
      // fixed automaton where its pattern stands, a union when the pattern
      // after its last one is reached (or at the end), a single right away.
      {
        std::vector<Group*> groups;
        for (auto& ch : packed)
          for (auto& g : ch) groups.push_back(&g);
        size_t gi = 0, left = 0;  // current group, its patterns not yet visited
        Group* open = nullptr;    // union waiting for its flush
        auto emit = [&](Group* g) {
          if (g->relaxed) relaxed_slots.push_back(g->ab.pes[0]->slot);
          if (g->always) P->always_slots.push_back(g->ab.pes[0]->slot);
          else autos.push_back(std::move(g->ab));
        };
        for (size_t pi = 0; pi < sb.pats.size(); pi++) {
          if (!is_union[pi]) {
            for (auto& ab : fixed[pi]) autos.push_back(std::move(ab));
            continue;
          }
          if (left == 0) {  // this pattern starts the next group
            if (open) emit(open);
            open = nullptr;
            Group* g = groups[gi++];
            left = g->n;
            if (g->unioned) open = g;
            else emit(g);
          }
          left--;
        }
        if (open) emit(open);
      }
      for (auto& u : unionable) owned.push_back(std::move(u.second));
      flush();
      // 1b. rune map: the joint partition of non-ASCII runes over the stream's
      // image automata.  Every rune of a joint class falls in one class of
      // each automaton, so k_stream can replace each non-ASCII rune of a value
      // by one byte 0x80 + joint class and k_scan steps once per rune through
      // the joint class map -- what the rune-decoding scan computes.  A stream
      // with a byte-mode automaton or more than 127 joint classes keeps its
      // non-ASCII values on the per-value path (k_scan_slow).
      std::vector<uint32_t> rmap;              // (lo, hi, joint class) triples
      std::vector<std::vector<uint8_t>> jcls;  // per joint class: the class in each automaton
      bool mappable = true;
      {
        auto cls_of = [](const Dfa& d, uint32_t r) -> uint8_t {
          const auto& nr = d.nranges;
          size_t lo = 0, hi = nr.size() / 3;
          while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (nr[mid * 3 + 1] < r) lo = mid + 1;
            else hi = mid;
          }
          return (lo < nr.size() / 3 && nr[lo * 3] <= r) ? (uint8_t)nr[lo * 3 + 2] : (uint8_t)0;
        };
        std::vector<uint32_t> bnd{0x80, 0x110000};
        for (const AutoBuild& ab : autos) {
          if (!img_ok(ab.d)) continue;
          if (ab.d.byte_mode) mappable = false;
          const auto& nr = ab.d.nranges;
          for (size_t i = 0; i + 2 < nr.size(); i += 3) {
            bnd.push_back(std::max<uint32_t>(nr[i], 0x80));
            bnd.push_back(std::min<uint32_t>(nr[i + 1] + 1, 0x110000));
          }
        }
        std::sort(bnd.begin(), bnd.end());
        bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
        std::map<std::vector<uint8_t>, uint32_t> ids;
        for (size_t i = 0; mappable && i + 1 < bnd.size(); i++) {
          if (bnd[i] >= 0x110000) break;
          std::vector<uint8_t> tup(autos.size(), 0);
          for (size_t k = 0; k < autos.size(); k++)
            if (img_ok(autos[k].d) && !autos[k].d.byte_mode) tup[k] = cls_of(autos[k].d, bnd[i]);
          auto it = ids.find(tup);
          uint32_t jc;
          if (it == ids.end()) {
            jc = (uint32_t)jcls.size();
            ids[tup] = jc;
            jcls.push_back(tup);
          } else {
            jc = it->second;
          }
          const uint32_t lo = bnd[i], hi = bnd[i + 1] - 1;
          if (!rmap.empty() && rmap[rmap.size() - 1] == jc && rmap[rmap.size() - 2] + 1 == lo) rmap[rmap.size() - 2] = hi;
          else rmap.insert(rmap.end(), {lo, hi, jc});
        }
        if (jcls.size() > 127) mappable = false;
      }
      // 2. stream record
      DStream s = sb.s;
      s.filt_begin = (uint32_t)P->sfilt.size();
      s.filt_count = (uint32_t)sb.filters.size();
      P->sfilt.insert(P->sfilt.end(), sb.gids.begin(), sb.gids.end());
      s.gmask = 0;
      for (uint8_t g : sb.gids) s.gmask |= 1ull << g;
      const uint32_t sid = (uint32_t)P->streams.size();
      s.val_begin = (uint32_t)P->svals.size();
      s.val_count = (uint32_t)sb.vals.size();
      P->svals.insert(P->svals.end(), sb.vals.begin(), sb.vals.end());
      s.job_begin = (uint32_t)P->jobs.size();
      s.collapse = mappable ? 1 : 0;  // values are rune-mapped (s.rmap_*) instead of going slow
      s.rmap_off = 0;
      s.rmap_cnt = 0;
      if (mappable && jcls.size() > 1) {  // one class: every non-ASCII rune -> GI_RUNE_MARK
        s.rmap_off = (uint32_t)P->nranges.size();
        s.rmap_cnt = (uint32_t)rmap.size() / 3;
        for (size_t i = 0; i < rmap.size(); i += 3) P->nranges.insert(P->nranges.end(), {rmap[i], rmap[i + 1], 0x80u + rmap[i + 2]});
      }
      s.det_id = 0xFF;
      for (const DScanVal& v : sb.vals)
        if (v.kind == OP_DETECT_SQLI || v.kind == OP_DETECT_XSS) {
          if (n_det >= GI_MAX_DET_STREAMS) unsup("more than 32 phase-A transformation chains with @detectSQLi/@detectXSS");
          s.det_id = (uint8_t)n_det++;
          break;
        }
      P->streams.push_back(s);
      if (!first_s) js << ",";
      first_s = false;
      js << "{\"chain\":[";
      for (uint32_t k = 0; k < s.tchain_len; k++) js << (k ? "," : "") << (int)P->tchains[s.tchain_off + k];
      js << "],\"kinds\":" << (int)s.kind_mask << ",\"filters\":[";
      for (uint32_t k = 0; k < s.filt_count; k++) {
        const DFilter& f = sb.filters[k];
        js << (k ? "," : "") << "{\"single\":" << (int)(f.single == GI_NO_SINGLE ? -1 : f.single)
           << ",\"kinds\":" << (int)f.kind_mask << ",\"names\":" << (int)f.names << ",\"key\":" << (int)f.key_mode
           << ",\"exc\":" << f.exc_count << "}";
      }
      js << "]"
         << ",\"vals\":" << sb.vals.size() << ",\"jobs\":[";
      // 3. jobs: pack up to GI_JOB_MAX_DFA automata per LDS image
      const uint32_t nf = (uint32_t)P->filters.size();  // fmask tables are indexed by global filter id
      size_t a = 0;
      bool first_j = true;
      while (a < autos.size()) {
        // choose the automata of this job
        std::vector<size_t> pick;
        bool lds = true;
        uint32_t need = GI_JAMAP_BYTES;
        while (a < autos.size() && pick.size() < GI_JOB_MAX_DFA) {
          const Dfa& d = autos[a].d;
          // a job holds prefix automata or others, not both (DJob.prefix)
          if (!pick.empty() && !autos[a].pes.empty() && !autos[pick[0]].pes.empty() &&
              pe_prefix(*autos[a].pes[0]) != pe_prefix(*autos[pick[0]].pes[0]))
            break;
          if (!img_ok(d)) {  // no image form: its patterns are always "maybe" (k_eval decides)
            for (const PatEntry* pe : autos[a].pes) P->always_slots.push_back(pe->slot);
            a++;
            continue;
          }
          if (!lds_ok(d, nf)) {
            if (pick.empty()) {  // image too large for LDS: its own job, image read from HBM
              pick.push_back(a++);
              lds = false;
            }
            break;
          }
          const uint32_t b = img_bytes(d) + al16(nf * 8) + al16(d.n_pat * 4);
          const uint32_t lim = pick.empty() ? GI_BIG_LDS_BYTES : GI_JOB_LDS_BYTES;
          if (need + b > lim) break;
          if (!pick.empty() && need + b > GI_JOB_LDS_BYTES) break;
          need += b;
          pick.push_back(a++);
        }
        if (pick.empty()) continue;
        DJob j{};
        j.stream = sid;
        j.img_off = (uint32_t)P->images.size();
        j.jdfa_begin = (uint32_t)P->jdfas.size();
        j.lds = lds ? 1 : 0;
        if (!first_j) js << ",";
        first_j = false;
        js << "[";
        std::vector<uint32_t> jam(GI_JAMAP_BYTES / 4, 0);
        int32_t at = 0;
        img_put(j.img_off, jam.data(), GI_JAMAP_BYTES, &at);  // filled below
        std::vector<uint32_t> slots;
        for (size_t q = 0; q < pick.size(); q++) {
          const AutoBuild& ab = autos[pick[q]];
          const Dfa& d = ab.d;
          DJobDfa jd{};
          jd.dfa = add_dfa(d);
          jd.lds_trans = jd.lds_amap = jd.lds_combo = jd.lds_endacc = jd.lds_slots = -1;
          {
            std::vector<uint16_t> tr(d.trans);
            if (!d.multi)  // absorbing accept row (already self-looping; made explicit)
              for (uint32_t c = 0; c < d.n_classes; c++) tr[(size_t)d.accept * d.n_classes + c] = (uint16_t)d.accept;
            img_put(j.img_off, tr.data(), tr.size() * 2, &jd.lds_trans);
            img_put(j.img_off, d.amap.data(), d.amap.size(), &jd.lds_amap);
            if (d.multi) {
              img_put(j.img_off, d.cls_combo.data(), d.cls_combo.size(), &jd.lds_combo);
              std::vector<uint64_t> em(d.n_states);
              for (uint32_t st = 0; st < d.n_states; st++) em[st] = d.acc[(size_t)st * 5 + 4];
              img_put(j.img_off, em.data(), em.size() * 8, &jd.lds_endacc);
            } else {
              img_put(j.img_off, d.end_accept.data(), d.end_accept.size(), &jd.lds_endacc);
            }
            for (uint32_t c = 0; c < 128; c++) jam[c] |= (uint32_t)d.amap[c] << (8 * q);
            // rune-mapped bytes 0x80 + joint class (stage 1b)
            for (size_t jc = 0; mappable && jc < jcls.size(); jc++) jam[0x80 + jc] |= (uint32_t)jcls[jc][pick[q]] << (8 * q);
            jd.lds_slots = (int32_t)(slots.size() * 4);  // relative; rebased below
          }
          jd.pat_begin = (uint32_t)P->pats.size();
          jd.n_pat = (uint32_t)ab.pes.size();
          jd.fmask_off = (uint32_t)P->u64pool.size();
          for (uint32_t fi = 0; fi < nf; fi++) P->u64pool.push_back(0);
          for (size_t k = 0; k < ab.pes.size(); k++) {
            const PatEntry* pe = ab.pes[k];
            P->pats.push_back(DPat{pe->slot});
            slots.push_back(pe->slot);
            if (pe->negate) jd.neg_mask |= 1ull << k;
            for (uint32_t fi = 0; fi < nf; fi++)
              if ((pe->fmask >> fi) & 1) P->u64pool[jd.fmask_off + fi] |= 1ull << k;
          }
          if (d.multi) P->n_union_dfas++;
          P->jdfas.push_back(jd);
          j.jdfa_count++;
          js << (q ? "," : "") << "{\"states\":" << d.n_states << ",\"classes\":" << d.n_classes
             << ",\"pats\":" << jd.n_pat << ",\"multi\":" << (d.multi ? 1 : 0) << ",\"lds\":" << (lds ? 1 : 0)
             << "}";
        }
        {
          memcpy(&P->images[j.img_off], jam.data(), GI_JAMAP_BYTES);
          std::vector<uint64_t> fm((size_t)j.jdfa_count * nf);
          for (uint32_t q = 0; q < j.jdfa_count; q++)
            for (uint32_t fi = 0; fi < nf; fi++) fm[(size_t)q * nf + fi] = P->u64pool[P->jdfas[j.jdfa_begin + q].fmask_off + fi];
          int32_t fo = 0, so = 0;
          img_put(j.img_off, fm.data(), fm.size() * 8, &fo);
          j.lds_fmask = (uint32_t)fo;
          img_put(j.img_off, slots.data(), slots.size() * 4, &so);
          for (uint32_t q = 0; q < j.jdfa_count; q++) P->jdfas[j.jdfa_begin + q].lds_slots += so;
        }
        js << "]";
        j.img_bytes = (uint32_t)(P->images.size() - j.img_off);
        j.big = j.img_bytes > GI_JOB_LDS_BYTES ? 1 : 0;
        if (lds) {
          if (j.big) P->max_big_img_bytes = std::max(P->max_big_img_bytes, j.img_bytes);
          else P->max_img_bytes = std::max(P->max_img_bytes, j.img_bytes);
        }
        P->jobs.push_back(j);
      }
      P->streams[sid].job_count = (uint32_t)P->jobs.size() - P->streams[sid].job_begin;
      js << "],\"collapse\":" << (int)P->streams[sid].collapse << ",\"rune_classes\":" << (mappable ? jcls.size() : 0)
         << "}";
    }
    js << "],\"jobs\":" << P->jobs.size() << ",\"hit_slots\":" << P->n_hit_slots
       << ",\"image_bytes\":" << P->images.size() << "}";
    P->plan_json = js.str();
    if (P->images.empty()) P->images.resize(16, 0);
  }

  uint32_t rule(const IrRule& r, bool child) {
    DRule d{};
    d.id = r.id;
    d.status = r.status;
    d.skip = r.skip;
    d.chain_next = -1;
    d.skip_after = r.skip_after.empty() ? -1 : marker(r.skip_after);
    d.marker = r.secmark.empty() ? -1 : marker(r.secmark);
    d.phase = (uint8_t)r.phase;
    d.flags = (child ? RF_CHILD : 0) | (r.secmark.empty() ? 0 : RF_MARKER);
    d.op = -1;
    const bool cap_obs = r.capture && r.has_op && (cap_global || cap_links.count(&r));
    if (cap_obs && r.op_name != "rx")
      unsup("capture on @" + r.op_name + " whose TX:0-TX:8 values a rule, macro or export reads");
    if (cap_obs && r.multimatch) unsup("observable capture with multiMatch");
    if (cap_obs) d.flags |= RF_CAPTURE;
    if (r.multimatch) d.flags |= RF_MULTIMATCH;
    const std::string& dis = r.disruptive;
    d.disruptive = dis == "deny" ? D_DENY : dis == "drop" ? D_DROP : dis == "redirect" ? D_REDIRECT
                   : dis == "pass" ? D_PASS : dis == "allow" ? D_ALLOW_ALL : dis == "allow:phase" ? D_ALLOW_PHASE
                   : dis == "allow:request" ? D_ALLOW_REQUEST : D_NONE;
    if (dis == "block") d.disruptive = D_NONE;  // block without a default disruptive action
    vars(r, &d);
    if (r.has_op) d.op = op(r);
    if (cap_obs) {  // the submatch program k_eval runs on every value the operator sees match
      Regex re;
      std::string err;
      if (!re_parse("(?sm)" + r.op_arg, &re, &err)) perr("invalid regex " + r.op_arg + ": " + err);
      DPike pk{};
      if (!build_pike(re, &P->pike_insts, &P->pike_ranges, &pk, &err)) unsup("capture: " + err);
      // CRS's "capture the whole value" idiom (920450 / 920451 on header names):
      // with (?s) the dot takes every rune, so group 0 is always [0, n)
      pk.whole = (r.op_arg == "^.*$" && pk.nslot == 2) ? 1u : 0u;
      P->pikes.push_back(pk);
      P->ops[d.op].pike = (int32_t)P->pikes.size() - 1;
      for (int g = 0; g < 9; g++) slot(std::to_string(g));  // TX.0-TX.8 (CaptureField keys)
    }
    d.tchain_off = (uint32_t)P->tchains.size();
    for (auto& t : r.transforms) {
      uint8_t code;
      transform_code(t, &code);
      P->tchains.push_back(code);
    }
    d.tchain_len = (uint32_t)P->tchains.size() - d.tchain_off;
    actions(r, &d);
    // a negated capturing link writes captures on values whose regex matches
    // -- exactly those that do not make the link match -- so it is always
    // evaluated by the interpreter (no phase-A bit)
    d.hit_slot = (cap_obs && r.op_neg) ? -1 : plan(r, d, &d.flags, &d.flags2);
    if (d.hit_slot >= 0 && pa_rx.count(&r)) d.flags2 |= RF2_PA_FILTER;
    P->rules.push_back(d);
    const uint32_t idx = (uint32_t)P->rules.size() - 1;
    if (d.hit_slot >= 0 && (d.flags & RF_RESIDUAL) && d.phase >= 2 && d.op >= 0)
      for (uint32_t vi = 0; vi < d.var_count; vi++)
        if (P->vars[d.var_begin + vi].var == S_REQUEST_BODY && P->vars[d.var_begin + vi].residual) {
          P->body_links.push_back(idx);
          std::stable_sort(P->body_links.begin(), P->body_links.end(), [&](uint32_t a, uint32_t b) {
            const DRule &x = P->rules[a], &y = P->rules[b];
            return std::lexicographical_compare(P->tchains.begin() + x.tchain_off,
                                                P->tchains.begin() + x.tchain_off + x.tchain_len,
                                                P->tchains.begin() + y.tchain_off,
                                                P->tchains.begin() + y.tchain_off + y.tchain_len);
          });
          break;
        }
    return idx;
  }
};

}  // namespace

// Rules phase A need not scan: those behind a CRS-style paranoia gate
//   SecRule TX:<X> "@lt N" "...,skipAfter:<M>"
// whose TX:<X> every setvar in the program sets to the same integer K < N.
// Such a region is skipped at run time for every request; dropping its links
// from phase A only saves scan work.  If a request does reach one (a ctl or
// a TX write this analysis does not see), the link has no hit slot and the
// interpreter evaluates it in full, so results never depend on the guess.
// Returns, per top-level rule, true = keep out of phase A.
static std::vector<bool> gated_rules(const IrWaf& waf) {
  std::vector<bool> out(waf.rules.size(), false);
  std::map<std::string, std::string> val;  // tx var -> integer text ("" = unknown)
  auto lower = [](std::string x) {
    for (auto& c : x) c = (char)tolower((unsigned char)c);
    return x;
  };
  auto is_int = [](const std::string& x) {
    if (x.empty()) return false;
    for (size_t i = (x[0] == '-' ? 1 : 0); i < x.size(); i++)
      if (!isdigit((unsigned char)x[i])) return false;
    return x != "-";
  };
  auto note = [&](const IrRule& r) {
    for (const IrNd& a : r.nd) {
      if (!a.is_setvar) {
        if (!a.ctl_name.empty()) val["*ctl"] = "";
        continue;
      }
      const std::string k = lower(a.sv_key);  // setvar keys are TX names (the "tx." is parsed off)
      std::string v = a.sv_remove ? std::string() : a.sv_value;
      if (v.size() > 5 && v.rfind("%{", 0) == 0 && v.back() == '}') {
        std::string ref = lower(v.substr(2, v.size() - 3));
        if (ref.rfind("tx.", 0) == 0 && val.count(ref.substr(3))) v = val[ref.substr(3)];
        else v = "";
      }
      if (!is_int(v) || v[0] == '+' || (val.count(k) && val[k] != v)) v = "";
      val[k] = v;
    }
  };
  for (const IrRule& r : waf.rules) {
    note(r);
    for (const IrRule& c : r.children) note(c);
  }
  std::map<std::string, size_t> marker_at;
  for (size_t i = 0; i < waf.rules.size(); i++)
    if (!waf.rules[i].secmark.empty()) marker_at[waf.rules[i].secmark] = i;
  for (size_t i = 0; i < waf.rules.size(); i++) {
    const IrRule& g = waf.rules[i];
    if (g.has_chain || g.skip_after.empty() || !g.has_op || g.op_neg || lower(g.op_name) != "lt" ||
        g.vars.size() != 1 || g.vars[0].count || g.vars[0].key_rx || lower(g.vars[0].name) != "tx")
      continue;
    auto it = val.find(lower(g.vars[0].key));
    auto mk = marker_at.find(g.skip_after);
    if (it == val.end() || it->second.empty() || !is_int(g.op_arg) || mk == marker_at.end() || mk->second <= i)
      continue;
    if (!(std::stoll(it->second) < std::stoll(g.op_arg))) continue;
    for (size_t j = i + 1; j < mk->second; j++)
      if (waf.rules[j].phase == g.phase) out[j] = true;
  }
  return out;
}

// `capture` (coraza internal/actions/capture.go; internal/operators/rx.go
// FindStringSubmatch -> TX.0-TX.8) changes nothing but the TX.0-TX.8 values:
// the operator's boolean result is the same with or without it.  A capture
// matters only if something reads those keys before the next capture
// overwrites them.  The analysis:
//   * readers: TX targets (a digit key, the whole collection, a regex key that
//     matches a digit key), %{tx.<digit>} macros (operator argument, setvar,
//     ctl), exported digit keys;
//   * a read of group k is "fed in chain" when a link of the reader's own
//     chain that certainly ran a capture of group k comes before the read:
//     a non-negated @rx with >= k groups (its chain successors only run when
//     it matched, and every match writes groups 0..ncap), or @detectSQLi for
//     k = 0.  For a target the feeder must be an earlier link; for an action
//     macro the link itself counts (its captures precede its actions); an
//     operator-argument macro is expanded before the link's own operator.
//   * if every read is fed in chain, the observable captures are those links
//     (the feeder and any capture link between it and the reader); otherwise
//     every capture in the program is observable (cap_global).
// CRS's capture rules are read only through logdata (not an output) except
// the 920420 / 920480 chains, which read their own parent's TX.0 / TX.1.
static void capture_analysis(const IrWaf& waf, const std::vector<std::string>& exports, bool* global,
                             std::set<const IrRule*>* links) {
  auto lowerc = [](std::string x) {
    for (auto& c : x) c = (char)tolower((unsigned char)c);
    return x;
  };
  auto digit_key = [](const std::string& k) { return k.size() == 1 && k[0] >= '0' && k[0] <= '9'; };
  // groups read by macros in s: bit k (bit 10: an unresolvable read)
  auto macro_groups = [&](const std::string& s) {
    uint32_t m = 0;
    const std::string l = lowerc(s);
    for (size_t p = l.find("%{"); p != std::string::npos; p = l.find("%{", p + 2)) {
      size_t q = p + 2;
      while (q < l.size() && (l[q] == ' ' || l[q] == '\t')) q++;
      if (l.compare(q, 2, "tx") == 0 && q + 3 < l.size() && (l[q + 2] == '.' || l[q + 2] == ':') &&
          isdigit((unsigned char)l[q + 3]))
        m |= (q + 4 < l.size() && isdigit((unsigned char)l[q + 4])) ? 0u : (1u << (l[q + 3] - '0'));
    }
    return m;
  };
  auto target_groups = [&](const IrRule& r) {
    uint32_t m = 0;
    for (const IrVar& v : r.vars) {
      if (lowerc(v.name) != "tx") continue;
      if (v.key.empty()) {
        m |= 0x3FFu;
      } else if (v.key_rx) {
        Regex re;
        std::string err;
        Dfa d;
        if (!re_parse(v.key, &re, &err) || !build_regex_dfa(re, &d, &err)) {
          m |= 0x3FFu;
        } else {
          for (int g = 0; g < 10; g++) {
            const uint8_t c = (uint8_t)('0' + g);
            if (dfa_host_match(d, &c, 1)) m |= 1u << g;
          }
        }
      } else if (digit_key(v.key)) {
        m |= 1u << (v.key[0] - '0');
      }
    }
    return m;
  };
  // groups link r certainly writes when it matched
  auto writes = [&](const IrRule& r) {
    if (!r.capture || !r.has_op || r.op_neg) return 0u;
    if (r.op_name == "detectsqli") return 1u;
    if (r.op_name != "rx") return 1u;  // @pm: at least TX.0 on a match
    Regex re;
    std::string err;
    if (!re_parse("(?sm)" + r.op_arg, &re, &err)) return 0u;
    return (1u << std::min(re.ncap + 1, 9)) - 1u;
  };
  *global = false;
  links->clear();
  for (const std::string& e : exports) {
    std::string k = lowerc(e);
    if (k.rfind("tx.", 0) == 0) k = k.substr(3);
    if (digit_key(k)) *global = true;
  }
  for (const IrRule& top : waf.rules) {
    std::vector<const IrRule*> chain{&top};
    for (const IrRule& c : top.children) chain.push_back(&c);
    for (size_t j = 0; j < chain.size(); j++) {
      const IrRule& r = *chain[j];
      uint32_t before = target_groups(r) | (r.has_op ? macro_groups(r.op_arg) : 0u);  // read before r's operator
      uint32_t after = 0;                                                              // read by r's actions
      for (const IrNd& a : r.nd) after |= macro_groups(a.sv_key) | macro_groups(a.sv_value) | macro_groups(a.ctl_value);
      for (int pass = 0; pass < 2; pass++) {
        const uint32_t need = pass == 0 ? before : after;
        const size_t last = pass == 0 ? j : j + 1;  // feeders: links [0, last)
        for (int g = 0; g < 10; g++) {
          if (!((need >> g) & 1u)) continue;
          if (g == 9) {  // TX.9 is never written by a capture: nothing to feed
            continue;
          }
          size_t f = last;
          while (f > 0 && !((writes(*chain[f - 1]) >> g) & 1u)) f--;
          if (f == 0) {
            *global = true;
            continue;
          }
          for (size_t x = f - 1; x < last; x++)
            if (chain[x]->capture) links->insert(chain[x]);
        }
      }
      if (((before | after) >> 10) & 1u) *global = true;
    }
  }
}

// ------------------------------------------ restricted-name chains (CRS 920450)
// CRS v4 920450 / 920451:
//   SecRule REQUEST_HEADERS_NAMES "@rx ^.*$" "capture,t:none,t:lowercase,
//       setvar:'tx.<P>%{tx.0}=/%{tx.0}/',chain"
//     SecRule TX:/^<P>/ "@within %{tx.<LIST>}" "..."
// The first link matches every name and files each one under a run-time TX
// key; the chain then asks whether some filed "/name/" is a substring of the
// list.  Phase A's "^.*$" bit is therefore set for every request with a
// header, and k_eval ran the capture, the macro-key setvar and the @within
// walk on every header of every request.  The chain can only match if some
// transformed name v has "/" + v + "/" inside a value LIST can hold, i.e. v is
// one of the finite set of strings between two '/' of that value.  When the
// keys <P>* and the capture are observable nowhere else, the names outside
// that set have no observable effect, so the first link's phase-A pattern
// becomes that set (exact): a clear bit skips the rule, and a set bit lets
// only the names in the set through field_filter (each still runs the link's
// capture and setvar in Coraza's order, so the chain sees the same keys it
// would have matched).  Conditions (anything else: no override):
//  * no capture group is observable outside its feeding chains (cap_global);
//  * the first link: @rx "^.*$", not negated, no multiMatch, transformations
//    t:none / t:lowercase ending in t:lowercase (so equal keys mean equal values), collection
//    targets only (no TX, no MATCHED_*, no counts), one setvar
//    'tx.<P>%{tx.0}=/%{tx.0}/' and no ctl, exactly one chained link;
//  * the chained link: TX:/^<P>/ with <P> a plain key literal, @within
//    "%{tx.<LIST>}", no transformation, capture or multiMatch;
//  * no other link, macro, setvar key or export can name a key starting with
//    <P> (so no other writer can interleave with the filed keys);
//  * no first link reads MATCHED_VAR / MATCHED_VAR_NAME (the names it skips
//    would otherwise have left them set);
//  * every setvar of <LIST> is a literal (the possible list values are those
//    literals and ""), ASCII, with at most 64 '/'.
// Returns first link -> the phase-A regex.
static std::map<const IrRule*, std::string> within_chain_filters(const IrWaf& waf,
                                                                  const std::vector<std::string>& exports,
                                                                  bool cap_global) {
  std::map<const IrRule*, std::string> out;
  if (cap_global) return out;
  auto lowerc = [](std::string x) {
    for (auto& c : x) c = (char)tolower((unsigned char)c);
    return x;
  };
  auto keychar = [](char c) { return isalnum((unsigned char)c) || c == '_' || c == '-' || c == '.'; };
  auto is_key_lit = [&](const std::string& s) {
    if (s.empty()) return false;
    for (char c : s)
      if (!keychar(c)) return false;
    return true;
  };
  // every TX key a macro in s reads, lowercased ("" when the key is not a plain literal)
  auto macro_keys = [&](const std::string& s) {
    std::vector<std::string> ks;
    const std::string l = lowerc(s);
    for (size_t p = l.find("%{"); p != std::string::npos; p = l.find("%{", p + 2)) {
      size_t q = p + 2;
      while (q < l.size() && (l[q] == ' ' || l[q] == '\t')) q++;
      if (l.compare(q, 2, "tx") != 0 || q + 2 >= l.size() || (l[q + 2] != '.' && l[q + 2] != ':')) continue;
      size_t e = q + 3;
      while (e < l.size() && keychar(l[e])) e++;
      ks.push_back(e < l.size() && l[e] == '}' ? l.substr(q + 3, e - q - 3) : std::string());
    }
    return ks;
  };
  auto reads_mv1 = [&](const std::string& s) {
    const std::string l = lowerc(s);
    for (size_t p = l.find("matched_var"); p != std::string::npos; p = l.find("matched_var", p + 1))
      if (l.compare(p, 12, "matched_vars") != 0) return true;
    return false;
  };
  std::vector<const IrRule*> links;
  for (const IrRule& t : waf.rules) {
    links.push_back(&t);
    for (const IrRule& c : t.children) links.push_back(&c);
  }
  // no first link may read MATCHED_VAR / MATCHED_VAR_NAME before its own match
  for (const IrRule& t : waf.rules) {
    for (const IrVar& v : t.vars) {
      const std::string n = lowerc(v.name);
      if (n == "matched_var" || n == "matched_var_name") return out;
    }
    if (t.has_op && reads_mv1(t.op_arg)) return out;
    if (!t.has_op)
      for (const IrNd& a : t.nd)
        if (reads_mv1(a.sv_key) || reads_mv1(a.sv_value) || reads_mv1(a.ctl_value)) return out;
  }
  const std::string m0 = "%{tx.0}";
  for (const IrRule& r : waf.rules) {
    if (!r.has_op || r.op_name != "rx" || r.op_neg || r.op_arg != "^.*$" || !r.capture || r.multimatch) continue;
    // t:lowercase last, and nothing but t:none / t:lowercase (k_eval records the
    // captures of the names the filter rejects by lowercasing them inline)
    bool lc_only = !r.transforms.empty() && lowerc(r.transforms.back()) == "lowercase";
    for (const auto& tf : r.transforms) lc_only = lc_only && (lowerc(tf) == "lowercase" || lowerc(tf) == "none");
    if (!lc_only) continue;
    if (r.children.size() != 1 || r.nd.size() != 1 || !r.nd[0].is_setvar || r.nd[0].sv_remove) continue;
    bool ok = !r.vars.empty();
    for (const IrVar& v : r.vars) {
      const std::string n = lowerc(v.name);
      if (v.count || n == "tx" || n.rfind("matched_var", 0) == 0 || single_id(v.name) >= 0) ok = false;
    }
    const std::string sk = lowerc(r.nd[0].sv_key), sv = lowerc(r.nd[0].sv_value);
    if (!ok || sk.size() <= m0.size() || sk.compare(sk.size() - m0.size(), m0.size(), m0) != 0 ||
        sv != "/" + m0 + "/")
      continue;
    const std::string pre = sk.substr(0, sk.size() - m0.size());
    if (!is_key_lit(pre)) continue;
    const IrRule& c = r.children[0];
    if (!c.has_op || c.op_name != "within" || c.op_neg || c.capture || c.multimatch || c.vars.size() != 1) continue;
    bool tnone = true;
    for (const auto& tf : c.transforms) tnone = tnone && lowerc(tf) == "none";
    const IrVar& cv = c.vars[0];
    if (!tnone || lowerc(cv.name) != "tx" || !cv.key_rx || cv.count || !cv.exc.empty() ||
        lowerc(cv.key) != "^" + pre)
      continue;
    const std::string ca = lowerc(trim(c.op_arg));
    if (ca.size() < 7 || ca.compare(0, 5, "%{tx.") != 0 || ca.back() != '}') continue;
    const std::string list = ca.substr(5, ca.size() - 6);
    if (!is_key_lit(list)) continue;
    // the keys <pre>* are named by nothing but r's setvar and c's target
    auto hits_pre = [&](const std::string& k) {  // a key (or key prefix) that can overlap <pre>*
      return k.compare(0, pre.size(), pre) == 0 || pre.compare(0, k.size(), k) == 0;
    };
    for (const std::string& e : exports) {
      std::string k = lowerc(e);
      if (k.rfind("tx.", 0) == 0) k = k.substr(3);
      if (k.compare(0, pre.size(), pre) == 0) ok = false;
    }
    std::set<std::string> values{""};  // what tx.<list> can hold
    std::set<std::string> extra;        // foreign key regexes a filed key can meet
    for (const IrRule* x : links) {
      if (!ok) break;
      for (const IrVar& v : x->vars) {
        if (lowerc(v.name) != "tx" || x == &c) continue;
        if (v.key.empty()) {
          ok = false;
        } else if (v.key_rx) {
          const std::string k = lowerc(v.key);
          if (k.size() > 1 && k[0] == '^' && is_key_lit(k.substr(1))) {
            if (hits_pre(k.substr(1))) ok = false;
            continue;
          }
          // an unanchored key regex F (CRS 921180's TX:/paramcounter_.*/) can match a
          // filed key <pre>v: when every match of F starts with a literal Lf that
          // neither occurs in <pre> nor starts inside it, and F has no context
          // assertion, F matches <pre>v iff it matches v -- so those names stay
          // visible too (the filter takes (?is:F) as well: a superset)
          size_t e = 0;
          while (e < k.size() && keychar(k[e]) && k[e] != '.') e++;
          const std::string lf = k.substr(0, e);
          bool straddle = lf.empty() || pre.find(lf) != std::string::npos;
          for (size_t q = 1; q < lf.size() && q <= pre.size() && !straddle; q++)
            if (pre.compare(pre.size() - q, q, lf, 0, q) == 0) straddle = true;  // Lf could start inside <pre>
          if (straddle || k.find('^') != std::string::npos || k.find("\\b") != std::string::npos ||
              k.find("\\B") != std::string::npos || k.find("\\A") != std::string::npos) {
            ok = false;
          } else {
            extra.insert(v.key);
          }
        } else if (lowerc(v.key).compare(0, pre.size(), pre) == 0) {
          ok = false;
        }
      }
      std::vector<std::string> srcs;
      if (x->has_op) srcs.push_back(x->op_arg);
      for (const IrNd& a : x->nd) {
        srcs.push_back(a.sv_value);
        srcs.push_back(a.ctl_value);
        if (!a.is_setvar) continue;
        const std::string k = lowerc(a.sv_key);
        const size_t mp = k.find("%{");
        if (x != &r) {
          if (mp == std::string::npos ? k.compare(0, pre.size(), pre) == 0 : hits_pre(k.substr(0, mp))) ok = false;
          srcs.push_back(a.sv_key);
        }
        // the list's writers: literal values only
        if (mp != std::string::npos ? list.compare(0, mp, k, 0, mp) == 0 : k == list) {
          if (mp != std::string::npos) {
            ok = false;
          } else if (a.sv_remove) {
            values.insert("");
          } else {
            const std::string& val = a.sv_value;
            if (val.find("%{") != std::string::npos || (!val.empty() && (val[0] == '+' || val[0] == '-'))) ok = false;
            values.insert(val);
          }
        }
      }
      for (const std::string& s : srcs)
        for (const std::string& k : macro_keys(s))
          if (k.empty() ? false : k.compare(0, pre.size(), pre) == 0) ok = false;
    }
    if (!ok) continue;
    // the strings between two '/' of a possible list value
    std::set<std::string> names;
    for (const std::string& val : values) {
      std::vector<size_t> sl;
      for (size_t i = 0; i < val.size(); i++) {
        if ((unsigned char)val[i] >= 0x80) ok = false;
        if (val[i] == '/') sl.push_back(i);
      }
      if (sl.size() > 64) ok = false;
      for (size_t a = 0; a < sl.size() && ok; a++)
        for (size_t b = a + 1; b < sl.size(); b++) names.insert(val.substr(sl[a] + 1, sl[b] - sl[a] - 1));
    }
    if (!ok) continue;
    std::vector<std::string> alts;
    if (!names.empty()) {
      std::string a = "^(?:";
      bool first = true;
      for (const std::string& n : names) {
        if (!first) a += "|";
        first = false;
        for (char ch : n) {
          if (ch && strchr("\\.+*?()|[]{}^$", ch)) a += '\\';
          a += ch;
        }
      }
      alts.push_back(a + ")$");
    }
    for (const std::string& f : extra) alts.push_back("(?is:" + f + ")");
    if (alts.empty()) continue;  // (the chain never matches and nothing else sees the keys: nothing to gain)
    std::string rx;
    for (const std::string& a : alts) rx += (rx.empty() ? "" : "|") + a;
    out[&r] = rx;
  }
  return out;
}

// ------------------------------------------------ constant folding
// CRS starts phase 1 with rules that read nothing but TX variables earlier
// rules set to constants (the 901 initialisation: `SecRule &TX:x "@eq 0"
// "setvar:tx.x=<default>"`), and gates every paranoia level on
// TX:DETECTION_PARANOIA_LEVEL.  Their outcomes are the same for every request,
// so the compiler evaluates them here, with the interpreter's semantics
// (kernels.hip eval_top / eval_rule / run_setvar / eval_op), instead of every
// k_eval lane re-evaluating them:
//   * prefix: the phase-1 walk from its start while every rule it reaches is
//     request-independent.  The TX state after it (tx_snap), the ids it
//     matched (fold_ids) and the walk index where evaluation resumes
//     (fold_walk) replace that stretch of the walk; k_eval reads TX slots from
//     the snapshot until the request writes them (copy on write).
//   * frozen slots: TX slots no rule outside the prefix can write (no setvar
//     names them, no capture group, no macro-key setvar whose literal key
//     prefix they start with).  A later request-independent link that reads
//     only frozen slots matches a fixed number of values (RF_CONST +
//     DRule._pad2); an operator argument that reads only frozen slots becomes
//     a literal.
// A link is request-independent when its targets are literal-key TX
// variables (or &count), it has no transformation, capture or ctl, its
// operator is a comparison / string test over literals and TX macros, and its
// actions are setvars over literals and TX macros.  Anything else stops the
// prefix (a ruleset that reads MATCHED_VAR / MATCHED_VAR_NAME, which the
// prefix's matches would set, gets no prefix).
namespace {
struct HSlot {
  uint32_t state = 0;  // 0 unset, 1 integer, 2 string
  int64_t num = 0;
  std::string s;
};

struct Folder {
  Program& P;
  std::vector<HSlot> tx;
  std::vector<bool> frozen;
  bool mv_single = false;   // MATCHED_VAR / MATCHED_VAR_NAME is read somewhere
  std::vector<std::pair<int64_t, int64_t>> rtgt_tx;  // ctl:ruleRemoveTargetById ranges naming TX

  explicit Folder(Program& p) : P(p), tx(p.n_slots), frozen(p.n_slots, false) {
    // MATCHED_VAR / MATCHED_VAR_NAME as an earlier rule left them are read by
    // those targets, by operator-argument macros (expanded before the link's
    // own matches) and by the actions of a link without targets; an action
    // macro of a link with targets reads the link's own match
    auto mv_parts = [&](int32_t tid) {
      if (tid < 0) return false;
      const DTmpl& tm = P.tmpls[tid];
      for (uint32_t k = 0; k < tm.part_count; k++) {
        const uint8_t kd = P.tparts[tm.part_begin + k].kind;
        if (kd == TP_MV || kd == TP_MVNAME) return true;
      }
      return false;
    };
    for (const DVarRef& v : P.vars)
      if (v.var == V_MATCHED_VAR || v.var == V_MATCHED_VAR_NAME) mv_single = true;
    for (const DRule& d : P.rules) {
      if (d.op >= 0 && mv_parts(P.ops[d.op].tmpl)) mv_single = true;
      if (d.var_count == 0)
        for (uint32_t k = 0; k < d.act_count; k++) {
          const DAction& a = P.acts[d.act_begin + k];
          if ((a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) && (mv_parts(a.tmpl) || (a.slot < 0 && mv_parts(a.aux))))
            mv_single = true;
        }
    }
    for (const DAction& a : P.acts)
      if (a.kind == A_CTL_RULE_REMOVE_TARGET && a.slot == V_TX) rtgt_tx.emplace_back(a.a, a.b);
  }
  static int64_t atoi0(const std::string& x) {
    int64_t v = 0;
    return go_atoi(x, &v) ? v : 0;
  }
  std::string slot_str(uint32_t sl) const {
    const HSlot& h = tx[sl];
    return h.state == 1 ? std::to_string(h.num) : h.state == 2 ? h.s : std::string();
  }
  bool slot_int(uint32_t sl, int64_t* v) const {
    const HSlot& h = tx[sl];
    if (h.state == 1) {
      *v = h.num;
      return true;
    }
    if (h.state == 2) return go_atoi(h.s, v);
    return false;
  }
  // template parts: literals and TX slots only (all frozen when `need_frozen`)
  bool tmpl_const(int tid, bool need_frozen) const {
    if (tid < 0) return true;
    const DTmpl& tm = P.tmpls[tid];
    for (uint32_t k = 0; k < tm.part_count; k++) {
      const DTmplPart& tp = P.tparts[tm.part_begin + k];
      if (tp.kind == TP_LIT) continue;
      if (tp.kind != TP_TX || tp.slot < 0) return false;
      if (need_frozen && !frozen[tp.slot]) return false;
    }
    return true;
  }
  std::string expand(int tid) const {
    std::string o;
    if (tid < 0) return o;
    const DTmpl& tm = P.tmpls[tid];
    for (uint32_t k = 0; k < tm.part_count; k++) {
      const DTmplPart& tp = P.tparts[tm.part_begin + k];
      if (tp.kind == TP_LIT) o.append((const char*)&P.strpool[tp.off], tp.len);
      else o += slot_str((uint32_t)tp.slot);
    }
    return o;
  }
  bool op_const(const DOp& o) const {
    switch (o.kind) {
      case OP_EQ: case OP_GE: case OP_GT: case OP_LE: case OP_LT: case OP_STREQ: case OP_WITHIN:
      case OP_BEGINSWITH: case OP_ENDSWITH: case OP_UNCONDITIONAL: case OP_NOMATCH:
        break;
      case OP_CONTAINS:
        if (o.dfa >= 0) return false;  // literal phrase automaton: not restated here
        break;
      default:
        return false;
    }
    return o.arg_is_lit || o.has_num || tmpl_const(o.tmpl, false);
  }
  // kernels.hip eval_op over a TX value
  bool eval_op(const DOp& o, const std::string& v) const {
    bool res = false;
    switch (o.kind) {
      case OP_UNCONDITIONAL: res = true; break;
      case OP_NOMATCH: res = false; break;
      case OP_EQ: case OP_GE: case OP_GT: case OP_LE: case OP_LT: {
        const int64_t a = o.has_num ? o.num : atoi0(expand(o.tmpl));
        const int64_t b = atoi0(v);
        res = o.kind == OP_EQ ? b == a : o.kind == OP_GE ? b >= a : o.kind == OP_GT ? b > a : o.kind == OP_LE ? b <= a : b < a;
        break;
      }
      default: {
        const std::string a = o.arg_is_lit ? std::string((const char*)&P.strpool[o.lit_off], o.lit_len) : expand(o.tmpl);
        switch (o.kind) {
          case OP_CONTAINS: res = v.find(a) != std::string::npos; break;
          case OP_STREQ: res = v == a; break;
          case OP_BEGINSWITH: res = v.size() >= a.size() && v.compare(0, a.size(), a) == 0; break;
          case OP_ENDSWITH: res = v.size() >= a.size() && v.compare(v.size() - a.size(), a.size(), a) == 0; break;
          case OP_WITHIN: res = a.find(v) != std::string::npos; break;
          default: break;
        }
      }
    }
    return o.negate ? !res : res;
  }
  // kernels.hip run_setvar
  void setvar(const DAction& a) {
    HSlot& sl = tx[(uint32_t)a.slot];
    if (a.kind == A_SETVAR_DEL) {
      sl.state = 0;
      return;
    }
    if (a.a == SV_SET_INT) {
      sl.state = 1;
      sl.num = a.b;
      return;
    }
    if (a.a != SV_GENERIC) {
      int64_t vv = a.b;
      bool generic = false;
      if (a.a == SV_ADD_SLOT || a.a == SV_SUB_SLOT) {
        const HSlot& src = tx[(uint32_t)a.b];
        if (src.state == 0) return;
        if (src.state != 1) generic = true;
        vv = src.num;
      }
      if (!generic) {
        int64_t me;
        if (!slot_int((uint32_t)a.slot, &me)) me = 0;
        const bool add = a.a == SV_ADD_CONST || a.a == SV_ADD_SLOT;
        sl.state = 1;
        sl.num = (int64_t)(add ? (uint64_t)me + (uint64_t)vv : (uint64_t)me - (uint64_t)vv);
        return;
      }
    }
    const std::string v = expand(a.tmpl);
    if (v.empty()) {
      sl.state = 2;
      sl.s.clear();
      return;
    }
    if (v[0] == '+' || v[0] == '-') {
      int64_t me;
      if (!slot_int((uint32_t)a.slot, &me)) me = 0;
      int64_t vv;
      if (!go_atoi(v.substr(1), &vv)) return;
      sl.state = 1;
      sl.num = (int64_t)(v[0] == '+' ? (uint64_t)me + (uint64_t)vv : (uint64_t)me - (uint64_t)vv);
      return;
    }
    int64_t num;
    if (go_atoi(v, &num) && std::to_string(num) == v) {
      sl.state = 1;
      sl.num = num;
      return;
    }
    sl.state = 2;
    sl.s = v;
  }
  bool tmpl_mv(int32_t tid) const {
    if (tid < 0) return false;
    const DTmpl& tm = P.tmpls[tid];
    for (uint32_t k = 0; k < tm.part_count; k++) {
      const uint8_t kd = P.tparts[tm.part_begin + k].kind;
      if (kd == TP_MV || kd == TP_MVNAME) return true;
    }
    return false;
  }
  // link ri's own actions or a later link of its chain read the matched-variable state
  bool chain_reads_mv(uint32_t ri) const {
    for (int32_t ci = (int32_t)ri; ci >= 0; ci = P.rules[ci].chain_next) {
      const DRule& d = P.rules[ci];
      for (uint32_t k = 0; k < d.act_count; k++) {
        const DAction& a = P.acts[d.act_begin + k];
        if ((a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) && (tmpl_mv(a.tmpl) || (a.slot < 0 && tmpl_mv(a.aux))))
          return true;
      }
      if ((uint32_t)ci == ri) continue;
      if (d.op >= 0 && tmpl_mv(P.ops[d.op].tmpl)) return true;
      for (uint32_t k = 0; k < d.var_count; k++)
        if (P.vars[d.var_begin + k].var >= V_MATCHED_VAR) return true;
    }
    return false;
  }
  // request-independent link (need_frozen: every TX slot it reads is frozen)
  bool link_ri(const DRule& d, bool need_frozen) const {
    if (d.flags & (RF_CAPTURE | RF_MARKER)) return false;
    if (d.tchain_len != 0) return false;
    if (d.op < 0 && d.var_count != 0) return false;
    if (d.op >= 0 && (d.var_count == 0 || !op_const(P.ops[d.op]))) return false;
    if (d.op >= 0 && need_frozen && !P.ops[d.op].arg_is_lit && !P.ops[d.op].has_num &&
        !tmpl_const(P.ops[d.op].tmpl, true))
      return false;
    for (uint32_t k = 0; k < d.var_count; k++) {
      const DVarRef& v = P.vars[d.var_begin + k];
      if (v.var != V_TX || v.key_mode != 1 || v.exc_count || v.slot < 0) return false;
      if (need_frozen && !frozen[v.slot]) return false;
    }
    for (const auto& rg : rtgt_tx)
      if (d.id != 0 && rg.first <= d.id && d.id <= rg.second) return false;
    for (uint32_t k = 0; k < d.act_count; k++) {
      const DAction& a = P.acts[d.act_begin + k];
      if (a.kind != A_SETVAR && a.kind != A_SETVAR_DEL) return false;
      if (a.slot < 0 || !tmpl_const(a.tmpl, false)) return false;
    }
    return true;
  }
  // kernels.hip eval_rule on a request-independent link: the number of values
  // it matches; apply: run the actions per match
  uint32_t eval_link(const DRule& d, bool apply) {
    if (d.op < 0) {
      if (apply)
        for (uint32_t k = 0; k < d.act_count; k++) setvar(P.acts[d.act_begin + k]);
      return 1;
    }
    const DOp& o = P.ops[d.op];
    uint32_t nm = 0;
    for (uint32_t k = 0; k < d.var_count; k++) {
      const DVarRef& v = P.vars[d.var_begin + k];
      std::string val;
      if (v.count) {
        val = tx[v.slot].state != 0 ? "1" : "0";
      } else {
        if (tx[v.slot].state == 0) continue;
        val = slot_str((uint32_t)v.slot);
      }
      if (eval_op(o, val)) {
        nm++;
        if (apply)
          for (uint32_t q = 0; q < d.act_count; q++) setvar(P.acts[d.act_begin + q]);
      }
    }
    return nm;
  }
};
}  // namespace

static void fold_program(Program* Pp, const std::vector<std::string>& exports) {
  (void)exports;
  Program& P = *Pp;
  Folder F(P);
  // the phase-1 walk (runtime.cpp load_program builds the same list)
  std::vector<uint32_t> walk;
  for (uint32_t ri : P.top)
    if (P.rules[ri].phase == 0 || P.rules[ri].phase == 1) walk.push_back(ri);
  std::vector<bool> in_prefix(P.rules.size(), false);  // links of folded rules
  std::vector<bool> fmatched(P.rules.size(), false);   // folded top-level rules that matched
  const uint32_t ns = P.n_slots;
  // the static TX slots a rule chain reads / writes
  std::vector<int32_t> dyn_site_of(P.acts.size(), -1);
  {
    int32_t di = 0;
    for (size_t q = 0; q < P.acts.size(); q++)
      if ((P.acts[q].kind == A_SETVAR || P.acts[q].kind == A_SETVAR_DEL) && P.acts[q].slot < 0) dyn_site_of[q] = di++;
  }
  auto slot_name = [&](uint32_t sl) {
    return std::string((const char*)&P.strpool[P.slot_names[2 * sl]], P.slot_names[2 * sl + 1]);
  };
  auto touch = [&](uint32_t top, std::vector<bool>& rd, std::vector<bool>& wr) {
    auto tmpl_reads = [&](int32_t tid) {
      if (tid < 0) return;
      const DTmpl& tm = P.tmpls[tid];
      for (uint32_t q = 0; q < tm.part_count; q++) {
        const DTmplPart& tp = P.tparts[tm.part_begin + q];
        if (tp.kind == TP_TX && tp.slot >= 0) rd[tp.slot] = true;
      }
    };
    for (int32_t ci = (int32_t)top; ci >= 0; ci = P.rules[ci].chain_next) {
      const DRule& d = P.rules[ci];
      for (uint32_t q = 0; q < d.var_count; q++) {
        const DVarRef& v = P.vars[d.var_begin + q];
        if (v.var != V_TX) continue;
        if (v.key_mode == 1 && v.slot >= 0) rd[v.slot] = true;
        else if (v.key_mode == 2)
          for (uint32_t j = 0; j < v.key_len; j++) rd[P.txrx[v.key_off + j]] = true;
        else if (v.key_mode == 0)
          for (uint32_t sl = 0; sl < ns; sl++) rd[sl] = true;
      }
      if (d.op >= 0) tmpl_reads(P.ops[d.op].tmpl);
      if (d.flags & RF_CAPTURE)
        for (uint32_t sl = 0; sl < ns; sl++) {
          const std::string nm = slot_name(sl);
          if (nm.size() == 1 && nm[0] >= '0' && nm[0] <= '9') wr[sl] = true;
        }
      for (uint32_t q = 0; q < d.act_count; q++) {
        const uint32_t ai = d.act_begin + q;
        const DAction& a = P.acts[ai];
        if (a.kind != A_SETVAR && a.kind != A_SETVAR_DEL) continue;
        tmpl_reads(a.tmpl);
        if ((a.a == SV_ADD_SLOT || a.a == SV_SUB_SLOT) && a.b >= 0) rd[a.b] = true;
        if (a.slot >= 0) {
          wr[a.slot] = true;
          rd[a.slot] = true;  // += reads it
        } else {
          tmpl_reads(a.aux);
          const DDynSite& ds = P.dyn_sites[dyn_site_of[ai]];
          const std::string pre((const char*)&P.strpool[ds.prefix_off], ds.prefix_len);
          for (uint32_t sl = 0; sl < ns; sl++)
            if (slot_name(sl).compare(0, pre.size(), pre) == 0) wr[sl] = rd[sl] = true;
        }
      }
    }
  };
  // a rule evaluated at run time that could keep a later folded rule from
  // running (or change its order): a skip, an interruption, ctl on the engine
  // or on rules
  auto barrier = [&](uint32_t top) {
    const DRule& R = P.rules[top];
    if (P.rule_engine == ENGINE_ON && R.disruptive != D_NONE && R.disruptive != D_PASS) return true;  // deny/drop/redirect/allow
    for (int32_t ci = (int32_t)top; ci >= 0; ci = P.rules[ci].chain_next) {
      const DRule& d = P.rules[ci];
      for (uint32_t q = 0; q < d.act_count; q++) {
        const uint8_t kd = P.acts[d.act_begin + q].kind;
        if (kd == A_CTL_RULE_ENGINE || kd == A_CTL_RULE_REMOVE_ID || kd == A_CTL_RULE_REMOVE_TARGET ||
            kd == A_CTL_RULE_REMOVE_GROUP)
          return true;
      }
    }
    return false;
  };
  // Fold every request-independent phase-1 rule that is reached by every
  // request and whose TX inputs / outputs no earlier run-time rule touches:
  // its effects are the snapshot (applied when phase 1 starts: a run-time rule
  // before it neither reads what it writes nor writes what it reads, so the
  // order does not matter), and its matched id is emitted where the walk
  // reaches it.  Consecutive folded rules (and the rules their skipAfter
  // jumps over) form a run: k_eval emits the run's ids and jumps past it.
  std::vector<bool> dep_r(ns, false), dep_w(ns, false);
  std::vector<bool> maybe_skipped(walk.size(), false);  // a run-time rule's skip / skipAfter may jump over it
  if (P.rule_engine != ENGINE_OFF) {
    int32_t skip_after = -1;
    int32_t skip = 0;
    int32_t run = -1;
    auto close_run = [&](uint32_t at) {
      if (run < 0) return;
      P.fold_runs[4 * run + 1] = (uint32_t)P.fold_ids.size() - P.fold_runs[4 * run];
      P.fold_runs[4 * run + 2] = at;
      P.fold_runs[4 * run + 3] = (uint32_t)skip_after;  // pending at the walk's end (else -1)
      run = -1;
    };
    uint32_t k = 0;
    for (; k < walk.size(); k++) {
      const uint32_t ri = walk[k];
      const DRule& R = P.rules[ri];
      if (skip_after >= 0) {  // inside a run: skipped for every request
        if (R.marker == skip_after) skip_after = -1;
        continue;
      }
      if (skip > 0) {
        skip--;
        continue;
      }
      if (R.flags & RF_MARKER) continue;
      bool ri_ok = !maybe_skipped[k];
      for (int32_t ci = (int32_t)ri; ri_ok && ci >= 0; ci = P.rules[ci].chain_next) {
        const DRule& C = P.rules[ci];
        ri_ok = F.link_ri(C, false) && !(F.mv_single && C.var_count);
      }
      if (ri_ok) {
        std::vector<bool> rd(ns, false), wr(ns, false);
        touch(ri, rd, wr);
        bool conflict = false;
        for (uint32_t sl = 0; sl < ns && !conflict; sl++)
          conflict = (rd[sl] && dep_w[sl]) || (wr[sl] && (dep_r[sl] || dep_w[sl]));
        if (!conflict) {
          const std::vector<HSlot> before = F.tx;
          bool matched = true;
          for (int32_t ci = (int32_t)ri; ci >= 0; ci = P.rules[ci].chain_next)
            if (F.eval_link(P.rules[ci], true) == 0) {
              matched = false;
              break;
            }
          const bool interrupts = matched && P.rule_engine == ENGINE_ON && R.disruptive != D_NONE &&
                                  R.disruptive != D_PASS;  // deny/drop/redirect, or allow (ends the walk)
          if (!interrupts) {
            for (int32_t ci = (int32_t)ri; ci >= 0; ci = P.rules[ci].chain_next) in_prefix[ci] = true;
            if (run < 0) {
              run = (int32_t)(P.fold_runs.size() / 4);
              P.fold_runs.insert(P.fold_runs.end(), {(uint32_t)P.fold_ids.size(), 0u, 0u, 0xFFFFFFFFu});
              P.rules[ri].flags |= RF_FOLDED;
              P.rules[ri]._pad2 = (uint32_t)run;
            }
            if (matched) {
              fmatched[ri] = true;
              if (R.skip_after >= 0) skip_after = R.skip_after;
              if (R.skip) skip = R.skip;
              if (R.id != 0) P.fold_ids.push_back((uint32_t)R.id);
            }
            continue;
          }
          F.tx = before;
        }
      }
      // evaluated at run time
      if (getenv("GI_FOLD_DEBUG"))
        fprintf(stderr, "fold: run-time rule %d at walk %u (ri_ok %d, barrier %d)\n", R.id, k, (int)ri_ok, (int)barrier(ri));
      close_run(k);
      if (barrier(ri)) break;
      touch(ri, dep_r, dep_w);
      // the entries its skip / skipAfter can jump over are not reached by every
      // request: they stay run-time rules (the walk continues after them)
      if (R.skip_after >= 0) {
        uint32_t m = k + 1;
        while (m < walk.size() && P.rules[walk[m]].marker != R.skip_after) m++;
        for (uint32_t j = k + 1; j < m && j < walk.size(); j++) maybe_skipped[j] = true;
      }
      for (uint32_t j = k + 1; j <= k + (uint32_t)std::max(R.skip, 0) && j < walk.size(); j++) maybe_skipped[j] = true;
    }
    close_run(k);
  }
  P.fold_on = P.fold_runs.empty() ? 0 : 1;
  if (!P.fold_on) {
    P.fold_ids.clear();
    for (auto& h : F.tx) h = HSlot();
  }
  // frozen slots: nothing outside the prefix writes them
  std::vector<bool> written(P.n_slots, false);
  for (uint32_t ri = 0; ri < P.rules.size(); ri++) {
    if (in_prefix[ri] && P.fold_on) continue;
    const DRule& d = P.rules[ri];
    for (uint32_t q = 0; q < d.act_count; q++) {
      const DAction& a = P.acts[d.act_begin + q];
      if ((a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) && a.slot >= 0) written[a.slot] = true;
    }
  }
  for (uint32_t sl = 0; sl < P.n_slots; sl++) {
    const std::string nm((const char*)&P.strpool[P.slot_names[2 * sl]], P.slot_names[2 * sl + 1]);
    bool w = written[sl];
    if (!P.pikes.empty() && nm.size() == 1 && nm[0] >= '0' && nm[0] <= '9') w = true;  // capture groups
    for (const DDynSite& ds : P.dyn_sites) {
      const std::string pre((const char*)&P.strpool[ds.prefix_off], ds.prefix_len);
      if (nm.compare(0, pre.size(), pre) == 0) w = true;  // a run-time key could name it
    }
    F.frozen[sl] = !w;
  }
  // links outside the prefix: constant outcomes, constant operator arguments
  uint32_t n_args = 0;
  if (P.rule_engine != ENGINE_OFF) {
    for (uint32_t ri = 0; ri < P.rules.size(); ri++) {
      if (in_prefix[ri] && P.fold_on) continue;
      DRule& d = P.rules[ri];
      if (d.op >= 0) {
        DOp& o = P.ops[d.op];
        if (!o.arg_is_lit && o.tmpl >= 0 && F.tmpl_const(o.tmpl, true)) {
          const std::string lit = F.expand(o.tmpl);
          o.arg_is_lit = 1;
          o.lit_off = (uint32_t)P.strpool.size();
          o.lit_len = (uint32_t)lit.size();
          P.strpool.insert(P.strpool.end(), lit.begin(), lit.end());
          P.strpool.push_back(0);
          int64_t v = 0;
          if (!go_atoi(lit, &v)) v = 0;
          o.has_num = 1;
          o.num = v;
          if (o.kind == OP_WITHIN) o.dfa = within_dfa(P.dfas, P.trans, P.u8pool, lit);
          n_args++;
        }
      }
      if (!F.link_ri(d, true)) continue;
      // the TX values it reads are the snapshot's for every request that reaches it
      const uint32_t nm = F.eval_link(d, false);
      // its matches would set the matched-variable state: fine unless a stale
      // reader exists (mv_single), or its own actions / later chain links read it
      if (nm > 0 && P.mv_used && (F.mv_single || F.chain_reads_mv(ri))) continue;
      d.flags |= RF_CONST;
      d._pad2 = nm;
    }
  }
  // Regions no request reaches: the rules between a constant gate (a rule whose
  // links all match for every request, RF_CONST / folded, with skipAfter:M,
  // that no ctl:ruleRemoveById can remove) and M, when no other rule's skip /
  // skipAfter can land inside.  Their matched-variable reads and macro-key
  // setvars then cost nothing: the per-request matched-variable state and
  // dynamic TX area are sized for the reachable rules only.
  std::vector<bool> dead(P.rules.size(), false);
  uint32_t n_mvcur = 0;  // chains recording MATCHED_VAR(_NAME) (RF2_MVCUR)
  if (P.rule_engine != ENGINE_OFF) {
    std::vector<std::pair<int64_t, int64_t>> removable;
    for (const DAction& a : P.acts)
      if (a.kind == A_CTL_RULE_REMOVE_ID) removable.emplace_back(a.a, a.b);
    for (int ph = 1; ph <= 2; ph++) {
      std::vector<uint32_t> w;
      for (uint32_t ri : P.top)
        if (P.rules[ri].phase == 0 || P.rules[ri].phase == (uint8_t)ph) w.push_back(ri);
      std::vector<uint32_t> mpos(P.n_markers, 0xFFFFFFFFu);  // first walk position of each marker
      for (uint32_t q = 0; q < w.size(); q++) {
        const int32_t m = P.rules[w[q]].marker;
        if (m >= 0 && mpos[m] == 0xFFFFFFFFu) mpos[m] = q;
      }
      for (uint32_t g = 0; g < w.size(); g++) {
        const DRule& G = P.rules[w[g]];
        if (G.skip_after < 0 || (G.flags & RF_MARKER)) continue;
        // every link matches for every request: constant links, or a folded rule that matched
        bool always = P.fold_on && in_prefix[w[g]] ? (bool)fmatched[w[g]] : true;
        for (int32_t ci = (int32_t)w[g]; always && ci >= 0 && !(P.fold_on && in_prefix[w[g]]); ci = P.rules[ci].chain_next)
          always = (P.rules[ci].flags & RF_CONST) && P.rules[ci]._pad2 > 0;
        if (!always) continue;
        for (const auto& rg : removable)
          if (G.id != 0 && rg.first <= G.id && G.id <= rg.second) always = false;
        if (P.n_rm_groups && P.rule_groups[w[g]]) always = false;
        const uint32_t me = G.skip_after < (int32_t)P.n_markers ? mpos[G.skip_after] : 0xFFFFFFFFu;
        if (!always || me == 0xFFFFFFFFu || me <= g + 1) continue;
        // nothing outside (g, me) lands inside it
        bool sealed = true;
        for (uint32_t q = 0; q < w.size() && sealed; q++) {
          if (q > g && q < me) continue;
          const DRule& Q = P.rules[w[q]];
          if (Q.skip_after >= 0 && Q.skip_after < (int32_t)P.n_markers && mpos[Q.skip_after] > g &&
              mpos[Q.skip_after] < me)
            sealed = false;
          if (Q.skip > 0 && q < g && q + (uint32_t)Q.skip >= g) sealed = false;
        }
        if (!sealed) continue;
        for (uint32_t q = g + 1; q < me; q++)
          for (int32_t ci = (int32_t)w[q]; ci >= 0; ci = P.rules[ci].chain_next) dead[ci] = true;
      }
    }
  }
  {  // matched-variable readers among the reachable rules
    bool mv = false;
    for (uint32_t ri = 0; ri < P.rules.size() && !mv; ri++) {
      if (dead[ri]) continue;
      const DRule& d = P.rules[ri];
      for (uint32_t q = 0; q < d.var_count; q++)
        if (P.vars[d.var_begin + q].var >= V_MATCHED_VAR) mv = true;
      if (d.op >= 0 && F.tmpl_mv(P.ops[d.op].tmpl)) mv = true;
      for (uint32_t q = 0; q < d.act_count; q++) {
        const DAction& a = P.acts[d.act_begin + q];
        if ((a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) && (F.tmpl_mv(a.tmpl) || (a.slot < 0 && F.tmpl_mv(a.aux))))
          mv = true;
      }
    }
    P.mv_used = mv ? 1 : 0;
    // MATCHED_VAR / MATCHED_VAR_NAME liveness: a chain's matches set them, and
    // only a later link of the same chain (or the link's own setvars) can read
    // what it set -- unless some reachable first link reads them before its
    // own match overwrites them (a MATCHED_VAR target, an operator argument or,
    // for a rule without operator, a setvar macro), in which case every chain
    // records them.  Chains whose values nobody reads skip the copies.
    bool first_reads = false;
    for (uint32_t ti : P.top) {
      if (dead[ti]) continue;
      const DRule& d = P.rules[ti];
      for (uint32_t q = 0; q < d.var_count; q++)
        if (P.vars[d.var_begin + q].var >= V_MATCHED_VAR) first_reads = true;
      if (d.op >= 0 && F.tmpl_mv(P.ops[d.op].tmpl)) first_reads = true;
      if (d.op < 0)
        for (uint32_t q = 0; q < d.act_count; q++) {
          const DAction& a = P.acts[d.act_begin + q];
          if ((a.kind == A_SETVAR || a.kind == A_SETVAR_DEL) && (F.tmpl_mv(a.tmpl) || (a.slot < 0 && F.tmpl_mv(a.aux))))
            first_reads = true;
        }
    }
    n_mvcur = 0;
    for (uint32_t ti : P.top)
      if (mv && (first_reads || F.chain_reads_mv(ti))) {
        P.rules[ti].flags2 |= RF2_MVCUR;
        n_mvcur++;
      }
  }
  {  // macro-key setvars in unreachable rules: no dynamic area for them
    std::vector<int32_t> site_rule(P.dyn_sites.size(), -1);
    uint32_t k = 0;
    for (uint32_t q = 0; q < P.acts.size(); q++)
      if ((P.acts[q].kind == A_SETVAR || P.acts[q].kind == A_SETVAR_DEL) && P.acts[q].slot < 0) {
        for (uint32_t ri = 0; ri < P.rules.size(); ri++)
          if (q >= P.rules[ri].act_begin && q < P.rules[ri].act_begin + P.rules[ri].act_count) site_rule[k] = (int32_t)ri;
        k++;
      }
    for (size_t q = 0; q < P.dyn_sites.size(); q++)
      if (site_rule[q] >= 0 && dead[site_rule[q]]) P.dyn_sites[q].dead = 1;
  }
  {  // the plan JSON reports what was folded
    uint32_t nconst = 0, nconst0 = 0;
    for (const DRule& d : P.rules)
      if (d.flags & RF_CONST) {
        nconst++;
        nconst0 += d._pad2 == 0;
      }
    uint32_t nfrozen = 0;
    for (bool f : F.frozen) nfrozen += f;
    uint32_t ndead = 0;
    for (bool x : dead) ndead += x;
    uint32_t nfold = 0;
    for (bool f : in_prefix) nfold += f;
    if (!P.plan_json.empty() && P.plan_json.back() == '}') {
      P.plan_json.pop_back();
      P.plan_json += ",\"fold\":{\"runs\":" + std::to_string(P.fold_runs.size() / 4) + ",\"folded_links\":" +
                     std::to_string(nfold) + ",\"ids\":" +
                     std::to_string(P.fold_ids.size()) + ",\"const_links\":" + std::to_string(nconst) +
                     ",\"const_nomatch\":" + std::to_string(nconst0) + ",\"const_args\":" + std::to_string(n_args) +
                     ",\"frozen_slots\":" + std::to_string(nfrozen) + ",\"dead_links\":" + std::to_string(ndead) +
                     ",\"mv_used\":" + std::to_string((int)P.mv_used) + ",\"mv_cur_chains\":" +
                     std::to_string(n_mvcur) + "}}";
    }
  }
  P.tx_snap.resize(P.n_slots);
  for (uint32_t sl = 0; sl < P.n_slots; sl++) {
    DSnapSlot z{};
    const HSlot& h = F.tx[sl];
    z.state = h.state;
    z.num = h.num;
    if (h.state == 2) {
      z.off = (uint32_t)P.strpool.size();
      z.len = (uint32_t)h.s.size();
      P.strpool.insert(P.strpool.end(), h.s.begin(), h.s.end());
      P.strpool.push_back(0);
    }
    P.tx_snap[sl] = z;
  }
  P.fold_nids = (uint32_t)P.fold_ids.size();
  if (P.fold_ids.empty()) P.fold_ids.push_back(0);  // a non-empty section (fold_nids is the count)
  if (P.fold_runs.empty()) P.fold_runs.insert(P.fold_runs.end(), {0u, 0u, 0u, 0xFFFFFFFFu});
}

int compile_program(const std::string& text, const std::vector<std::string>& exports, uint32_t cap,
                    Program* out, std::string* err, const std::map<std::string, std::string>* data_files) {
  struct FilesScope {
    explicit FilesScope(const std::map<std::string, std::string>* f) { g_data_files = f; }
    ~FilesScope() { g_data_files = nullptr; }
  } files_scope(data_files);
  const bool timing = getenv("GI_COMPILE_TIMING") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "gi_compile: %-16s %8.3f s\n", what, std::chrono::duration<double>(now - t_prev).count());
    t_prev = now;
  };
  try {
    IrWaf waf = parse_seclang(text);
    lap("parse");
    Lower L;
    L.P = out;
    L.cap = cap ? cap : 60000;
    *out = Program();
    // block inherits the phase's default disruptive action through merge_defaults:
    // the merged list then holds "block" followed by the default action; the last
    // disruptive action wins (apply_actions), so nothing else is needed here.
    const std::vector<bool> gated = gated_rules(waf);
    capture_analysis(waf, exports, &L.cap_global, &L.cap_links);
    static const bool pa_filter_env = !(getenv("GI_PA_FILTER") && atoi(getenv("GI_PA_FILTER")) == 0);  // A/B knob
    if (pa_filter_env) L.pa_rx = within_chain_filters(waf, exports, L.cap_global);
    if (timing) fprintf(stderr, "gi_compile: captures observable globally: %d\n", (int)L.cap_global);
    if (timing)
      for (const auto& kv : L.pa_rx)
        fprintf(stderr, "gi_compile: rule %d: phase-A filter %zu bytes\n", kv.first->id, kv.second.size());
    for (size_t ti = 0; ti < waf.rules.size(); ti++) {
      const IrRule& r = waf.rules[ti];
      L.no_scan = gated[ti];
      uint32_t idx = L.rule(r, false);
      out->top.push_back(idx);
      uint32_t prev = idx;
      for (auto& c : r.children) {
        uint32_t ci = L.rule(c, true);
        out->rules[prev].chain_next = (int32_t)ci;
        prev = ci;
      }
    }
    lap("lower rules");
    // chains whose evaluation over a body needs the body's phase-A scan (RF2_BODY_PA)
    for (uint32_t ti : out->top)
      for (int32_t ci = (int32_t)ti; ci >= 0; ci = out->rules[ci].chain_next) {
        const DRule& d = out->rules[ci];
        if (d.op < 0) continue;
        const uint8_t k = out->ops[d.op].kind;
        if (k != OP_RX && k != OP_PM && k != OP_CONTAINS && k != OP_CONTAINSWORD && k != OP_DETECT_SQLI &&
            k != OP_DETECT_XSS)
          continue;
        bool body = false;
        for (uint32_t q = 0; q < d.var_count && !body; q++) {
          const uint8_t v = out->vars[d.var_begin + q].var;
          // (REQUEST_BODY: k_body's bits, computed in the gate's first stage)
          body = v == V_ARGS_POST || v == V_ARGS || v == V_ARGS_POST_NAMES ||
                 v == V_ARGS_NAMES || v == V_XML || v == V_FILES || v == V_FILES_NAMES || v == V_FILES_SIZES ||
                 v == V_FILES_TMPNAMES || v == V_MULTIPART_PART_HEADERS;
        }
        if (body) {
          out->rules[ti].flags2 |= RF2_BODY_PA;
          break;
        }
      }
    // the gate's prefix links: those of the phase-2 rules before the first RF2_BODY_PA rule
    {
      for (uint32_t ti : out->top) {
        if (out->rules[ti].phase != 2) continue;
        if (out->rules[ti].flags2 & RF2_BODY_PA) {
          if (timing) fprintf(stderr, "gi_compile: gate prefix ends at rule %d\n", out->rules[ti].id);
          break;
        }
        for (int32_t ci = (int32_t)ti; ci >= 0; ci = out->rules[ci].chain_next) out->rules[ci].flags2 |= RF2_PREFIX;
      }
    }
    L.finish_streams();
    {  // a phase-A hit of a relaxed automaton is never an exact match (field_filter re-runs the operator)
      std::vector<char> rel(out->n_hit_slots, 0);
      for (uint32_t sl : L.relaxed_slots)
        if (sl < rel.size()) rel[sl] = 1;
      for (DRule& d : out->rules)
        if (d.hit_slot >= 0 && (uint32_t)d.hit_slot < rel.size() && rel[d.hit_slot]) d.flags2 |= RF2_PA_RELAXED;
    }
    lap("scan plan");
    // ctl removal groups: each top-level rule's membership (its tags / msg)
    out->n_rm_groups = (uint32_t)L.rm_groups.size();
    out->rule_groups.assign(std::max<size_t>(out->rules.size(), 1), 0u);
    if (out->n_rm_groups)
      for (size_t ti = 0; ti < waf.rules.size(); ti++) {
        const IrRule& r = waf.rules[ti];
        uint32_t m = 0;
        for (const auto& g : L.rm_groups) {
          const bool tag = g.first[0] == 't';
          const std::string v = g.first.substr(2);
          if (tag ? std::find(r.tags.begin(), r.tags.end(), v) != r.tags.end() : (r.secmark.empty() && r.msg == v))
            m |= 1u << g.second;
        }
        out->rule_groups[out->top[ti]] = m;
      }
    out->args_limit = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(waf.args_limit, 0x7FFFFFFF));
    // chains whose later links read MATCHED_VARS(_NAMES) (the first link reads
    // them right after RuleGroup.Eval's reset: empty)
    for (uint32_t ti : out->top)
      for (int32_t ci = out->rules[ti].chain_next; ci >= 0; ci = out->rules[ci].chain_next)
        for (uint32_t q = 0; q < out->rules[ci].var_count; q++)
          if (out->vars[out->rules[ci].var_begin + q].var == V_MATCHED_VARS ||
              out->vars[out->rules[ci].var_begin + q].var == V_MATCHED_VARS_NAMES)
            out->rules[ti].flags2 |= RF2_MVS;
    // the gate's prefix: the links of the phase-2 rules before the first RF2_BODY_PA
    // rule, and every phase-A stream one of them registered a pattern / value test in
    {
      std::vector<int32_t> slot_link(out->n_hit_slots, -1);
      for (size_t ri = 0; ri < out->rules.size(); ri++)
        if (out->rules[ri].hit_slot >= 0 && (uint32_t)out->rules[ri].hit_slot < out->n_hit_slots)
          slot_link[out->rules[ri].hit_slot] = (int32_t)ri;
      auto prefix_slot = [&](uint32_t sl) {
        return sl < slot_link.size() && slot_link[sl] >= 0 && (out->rules[slot_link[sl]].flags2 & RF2_PREFIX);
      };
      for (DScanVal& v : out->svals) v.prefix = prefix_slot(v.slot) ? 1 : 0;
      for (DJob& J : out->jobs) {
        bool pre = false;
        for (uint32_t q = 0; q < J.jdfa_count && !pre; q++) {
          const DJobDfa& jd = out->jdfas[J.jdfa_begin + q];
          for (uint32_t k = 0; k < jd.n_pat && !pre; k++) pre = prefix_slot(out->pats[jd.pat_begin + k].slot);
        }
        J.prefix = pre ? 1 : 0;
      }
      for (DStream& st : out->streams) {
        bool pre = false;
        for (uint32_t q = 0; q < st.val_count; q++) pre = pre || out->svals[st.val_begin + q].prefix;
        for (uint32_t j = 0; j < st.job_count; j++) pre = pre || out->jobs[st.job_begin + j].prefix;
        st.prefix = pre ? 1 : 0;
      }
      if (timing) {
        uint32_t np = 0, nl = 0, nj = 0;
        for (const DStream& st : out->streams) np += st.prefix;
        for (const DJob& J : out->jobs) nj += J.prefix;
        for (const DRule& d : out->rules) nl += (d.flags2 & RF2_PREFIX) ? 1 : 0;
        fprintf(stderr, "gi_compile: gate prefix: %u links, %u of %zu streams, %u of %zu jobs\n", nl, np,
                out->streams.size(), nj, out->jobs.size());
      }
    }
    {  // top-level rules with an observable capture link (capture records, gi_capture)
      std::string ids;
      for (uint32_t ti : out->top)
        for (int32_t ci = (int32_t)ti; ci >= 0; ci = out->rules[ci].chain_next)
          if (out->rules[ci].flags & RF_CAPTURE) {
            ids += (ids.empty() ? "" : ",") + std::to_string(out->rules[ti].id);
            break;
          }
      out->plan_json.pop_back();  // the closing brace
      out->plan_json += ",\"capture_rules\":[" + ids + "]}";
    }
    if (out->u64pool.empty()) out->u64pool.push_back(0);
    out->rule_engine = waf.engine == "On" ? ENGINE_ON : waf.engine == "Off" ? ENGINE_OFF : ENGINE_DETECTION_ONLY;
    out->body_access = waf.body_access;
    out->body_limit = (uint64_t)waf.body_limit;
    out->body_partial = waf.body_partial ? 1 : 0;
    out->export_names = exports;
    for (auto& e : exports) out->exports.push_back(L.slot(e));
    out->n_slots = (uint32_t)L.slots.size();
    out->n_markers = (uint32_t)L.markers.size();
    // regex-keyed TX targets: the static slots whose (lowercase) names the key
    // regex matches, listed once here instead of matched per request; keys a
    // macro-key setvar creates at run time are matched by k_eval
    for (const auto& tv : L.tx_rx_vars) {
      DVarRef& v = out->vars[tv.first];
      Regex re;
      Dfa d;
      std::string e2;
      if (!re_parse(tv.second, &re, &e2) || !build_regex_dfa(re, &d, &e2, L.cap))
        unsup("TX key regex " + tv.second + ": " + e2);
      v.key_off = (uint32_t)out->txrx.size();
      for (uint32_t sidx = 0; sidx < out->n_slots; sidx++) {
        const uint8_t* nm = &out->strpool[out->slot_names[2 * sidx]];
        if (dfa_host_match(d, nm, out->slot_names[2 * sidx + 1])) out->txrx.push_back(sidx);
      }
      v.key_len = (uint32_t)out->txrx.size() - v.key_off;
    }
    if (out->txrx.empty()) out->txrx.push_back(0);
    lap("tx regex keys");
    fold_program(out, exports);
    lap("fold");
    for (const DAction& a : out->acts)  // literal setvar values (snapshot strings are literals or their expansions)
      if ((a.kind == A_SETVAR) && a.tmpl >= 0) {
        const DTmpl& tm = out->tmpls[a.tmpl];
        uint32_t n = 0;
        for (uint32_t k = 0; k < tm.part_count; k++)
          if (out->tparts[tm.part_begin + k].kind == TP_LIT) n += out->tparts[tm.part_begin + k].len;
        out->max_tx_lit = std::max(out->max_tx_lit, n);
      }
    for (const DSnapSlot& z : out->tx_snap) out->max_tx_lit = std::max(out->max_tx_lit, z.len);
    if (out->strpool.empty()) out->strpool.push_back(0);
    if (out->u8pool.empty()) out->u8pool.push_back(0);
    if (out->trans.empty()) out->trans.push_back(0);
    if (out->nranges.empty()) out->nranges.push_back(0);
    if (out->tchains.empty()) out->tchains.push_back(0);
    if (out->slot_names.empty()) out->slot_names.push_back(0);
    return 0;
  } catch (const CompileError& e) {
    *err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    *err = std::string("internal compiler error: ") + e.what();
    return -2;
  }
}

}  // namespace gi
