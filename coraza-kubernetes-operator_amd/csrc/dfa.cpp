// Thompson NFA -> rune-class DFA (single sticky or multi-pattern union),
// Aho-Corasick phrase automata, and the host self-test walker.
// See regex.h for the automaton contracts.
#include <algorithm>
#include <queue>
#include <unordered_map>

#include "regex.h"

namespace gi {
namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;
const RuneSet kWord = {{0x30, 0x39}, {0x41, 0x5A}, {0x5F, 0x5F}, {0x61, 0x7A}};
const RuneSet kNl = {{'\n', '\n'}};

enum InstOp : uint8_t { I_CLASS, I_SPLIT, I_EMPTY, I_MATCH, I_NOP };
struct Inst {
  InstOp op;
  int out = -1, out1 = -1;
  uint8_t assert_kind = 0;
  int arg = -1;  // I_CLASS: class-set id; I_MATCH: pattern index
};
struct Frag {
  int start;
  std::vector<std::pair<int, int>> outs;  // (inst, which)
};

struct NfaBuilder {
  const Regex& re;
  std::vector<Inst>& prog;
  const std::vector<int>& node_cset;  // node index -> class-set id (N_CLASS)
  size_t cap;
  bool overflow = false;

  NfaBuilder(const Regex& r, std::vector<Inst>& p, const std::vector<int>& nc, size_t c)
      : re(r), prog(p), node_cset(nc), cap(c) {}

  int emit(Inst in) {
    if (prog.size() >= cap) overflow = true;
    prog.push_back(in);
    return (int)prog.size() - 1;
  }
  void patch(const std::vector<std::pair<int, int>>& outs, int to) {
    for (auto& o : outs) (o.second == 0 ? prog[o.first].out : prog[o.first].out1) = to;
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
        in.arg = node_cset[id];
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
          // x{m,} = x{m-1} x+
          Frag last = plus(compile(sub));
          if (n.min == 1) return last;
          Frag f = compile(sub);
          for (int k = 1; k < n.min - 1; k++) f = cat(std::move(f), compile(sub));
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
        if (n.max > n.min) {
          Frag opt = quest(compile(sub));
          for (int k = n.min + 1; k < n.max; k++) {
            Frag c = compile(sub);
            Frag inner = cat(std::move(c), std::move(opt));
            opt = quest(std::move(inner));
          }
          f = have ? cat(std::move(f), std::move(opt)) : std::move(opt);
        }
        return f;
      }
    }
    return nop();
  }
};

// Moore partition refinement.  Single: blocks start from {accept, end_accept};
// multi: from the 5 accept masks; transitions compare (target block, flag).
void minimize(Dfa* d) {
  const uint32_t n = d->n_states, k = d->n_classes;
  std::vector<uint32_t> block(n);
  {
    std::unordered_map<std::string, uint32_t> init;
    for (uint32_t s = 0; s < n; s++) {
      std::string key;
      if (d->multi) {
        key.assign((const char*)&d->acc[(size_t)s * 5], 5 * sizeof(uint64_t));
      } else {
        key.push_back(s == d->accept ? 'A' : 'n');
        key.push_back((char)d->end_accept[s]);
      }
      auto it = init.find(key);
      if (it == init.end()) it = init.emplace(key, (uint32_t)init.size()).first;
      block[s] = it->second;
    }
  }
  uint32_t nblocks = 0;
  for (;;) {
    std::unordered_map<std::string, uint32_t> sig;
    std::vector<uint32_t> nb(n);
    std::string key;
    for (uint32_t s = 0; s < n; s++) {
      key.assign((const char*)&block[s], 4);
      for (uint32_t c = 0; c < k; c++) {
        uint16_t t = d->trans[(size_t)s * k + c];
        uint32_t v = block[t & 0x7FFF] | ((uint32_t)(t & 0x8000) << 16);
        key.append((const char*)&v, 4);
      }
      auto it = sig.find(key);
      if (it == sig.end()) it = sig.emplace(key, (uint32_t)sig.size()).first;
      nb[s] = it->second;
    }
    uint32_t cnt = (uint32_t)sig.size();
    block.swap(nb);
    if (cnt == nblocks) break;
    nblocks = cnt;
  }
  std::vector<int> newid(nblocks, -1);
  uint32_t next = 0;
  newid[block[d->start]] = next++;
  if (!d->multi && newid[block[d->accept]] < 0) newid[block[d->accept]] = next++;
  for (uint32_t s = 0; s < n; s++)
    if (newid[block[s]] < 0) newid[block[s]] = next++;
  std::vector<uint16_t> tr((size_t)nblocks * k);
  std::vector<uint8_t> ea(nblocks);
  std::vector<uint64_t> acc(d->multi ? (size_t)nblocks * 5 : 0);
  for (uint32_t s = 0; s < n; s++) {
    uint32_t b = newid[block[s]];
    ea[b] = d->end_accept[s];
    if (d->multi)
      for (int j = 0; j < 5; j++) acc[(size_t)b * 5 + j] = d->acc[(size_t)s * 5 + j];
    for (uint32_t c = 0; c < k; c++) {
      uint16_t t = d->trans[(size_t)s * k + c];
      tr[(size_t)b * k + c] = (uint16_t)(newid[block[t & 0x7FFF]] | (t & 0x8000));
    }
  }
  d->start = newid[block[d->start]];
  if (!d->multi) d->accept = newid[block[d->accept]];
  d->n_states = nblocks;
  d->trans.swap(tr);
  d->end_accept.swap(ea);
  d->acc.swap(acc);
}

// Rune-class partition over every set of every pattern + word chars + '\n':
// the alphabet of both the DFA and the NFA tables.
struct ClassPart {
  std::vector<std::vector<int>> node_set;  // per pattern: node -> class-set id
  uint32_t ncls = 0;
  std::vector<uint8_t> amap;                // 128 ASCII entries
  std::vector<uint32_t> nranges;            // (lo, hi, cls) for runes >= 0x80
  std::vector<uint8_t> cls_combo;           // bit0 '\n', bit1 word char
  std::vector<std::vector<uint64_t>> set_bits;  // class-set id -> classes it holds
  uint32_t cls_nl = 0;
  std::vector<uint8_t> cls_word;
};

bool partition_classes(const std::vector<const Regex*>& pats, ClassPart* cp, std::string* err) {
  std::vector<const RuneSet*> sets = {&kWord, &kNl};
  std::vector<std::vector<int>>& node_set = cp->node_set;
  node_set.assign(pats.size(), {});
  {
    std::unordered_map<std::string, int> uniq;
    for (size_t p = 0; p < pats.size(); p++) {
      const Regex& re = *pats[p];
      node_set[p].assign(re.nodes.size(), -1);
      for (size_t i = 0; i < re.nodes.size(); i++) {
        if (re.nodes[i].kind != N_CLASS) continue;
        std::string key((const char*)re.nodes[i].set.data(), re.nodes[i].set.size() * sizeof(RuneRange));
        auto it = uniq.find(key);
        if (it == uniq.end()) {
          sets.push_back(&re.nodes[i].set);
          it = uniq.emplace(key, (int)sets.size() - 1).first;
        }
        node_set[p][i] = it->second;
      }
    }
  }
  std::vector<uint32_t> bounds = {0, kMaxRune + 1};
  for (auto* s : sets)
    for (auto& r : *s) {
      bounds.push_back(r.lo);
      bounds.push_back(r.hi + 1);
    }
  for (uint32_t c = 0; c <= 0x80; c++) bounds.push_back(c);
  std::sort(bounds.begin(), bounds.end());
  bounds.erase(std::unique(bounds.begin(), bounds.end()), bounds.end());
  const size_t nsets = sets.size();
  std::vector<size_t> cursor(nsets, 0);
  std::unordered_map<std::string, uint32_t> sigmap;
  std::vector<std::string> class_sig;
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
      it = sigmap.emplace(sig, (uint32_t)class_sig.size()).first;
      class_sig.push_back(sig);
    }
    interval_class.push_back(it->second);
  }
  const uint32_t ncls = (uint32_t)class_sig.size();
  if (ncls > 255) {
    *err = "automaton needs more than 255 rune classes";
    return false;
  }
  cp->ncls = ncls;
  cp->amap.assign(128, 0);
  for (size_t b = 0; b + 1 < bounds.size(); b++) {
    uint32_t lo = bounds[b], hi = bounds[b + 1] - 1;
    if (lo < 0x80) {
      for (uint32_t c = lo; c <= hi && c < 0x80; c++) cp->amap[c] = (uint8_t)interval_class[b];
    } else {
      uint32_t cl = interval_class[b];
      size_t m = cp->nranges.size();
      if (m >= 3 && cp->nranges[m - 1] == cl && cp->nranges[m - 2] + 1 == lo) {
        cp->nranges[m - 2] = hi;
      } else {
        cp->nranges.push_back(lo);
        cp->nranges.push_back(hi);
        cp->nranges.push_back(cl);
      }
    }
  }
  const uint32_t cls_nl = cp->amap['\n'];
  cp->cls_nl = cls_nl;
  std::vector<uint8_t>& cls_word = cp->cls_word;
  cls_word.assign(ncls, 0);
  for (uint32_t c = 0; c < ncls; c++) cls_word[c] = (uint8_t)class_sig[c][0];
  cp->cls_combo.assign(ncls, 0);
  for (uint32_t c = 0; c < ncls; c++) cp->cls_combo[c] = (c == cls_nl ? 1 : 0) | (cls_word[c] ? 2 : 0);
  const size_t words = (ncls + 63) / 64;
  std::vector<std::vector<uint64_t>>& set_bits = cp->set_bits;
  set_bits.assign(nsets, std::vector<uint64_t>(words, 0));
  for (uint32_t c = 0; c < ncls; c++)
    for (size_t si = 0; si < nsets; si++)
      if (class_sig[c][si]) set_bits[si][c >> 6] |= 1ull << (c & 63);

  return true;
}

// Shared subset construction over a list of patterns.
bool build_core(const std::vector<const Regex*>& pats, bool multi, Dfa* out, std::string* err,
                uint32_t state_cap, uint32_t byte_budget = 0) {
  *out = Dfa();
  out->multi = multi;
  out->n_pat = (uint32_t)pats.size();
  if (multi && pats.size() > 64) {
    *err = "too many patterns for one union automaton";
    return false;
  }
  ClassPart cp;
  if (!partition_classes(pats, &cp, err)) return false;
  const std::vector<std::vector<int>>& node_set = cp.node_set;
  const uint32_t ncls = cp.ncls;
  if (byte_budget) state_cap = std::min<uint32_t>(state_cap, byte_budget / (2 * ncls + (multi ? 8 : 1)) + 1);
  out->n_classes = ncls;
  out->amap = cp.amap;
  out->nranges = cp.nranges;
  out->cls_combo = cp.cls_combo;
  const uint32_t cls_nl = cp.cls_nl;
  const std::vector<uint8_t>& cls_word = cp.cls_word;
  const std::vector<std::vector<uint64_t>>& set_bits = cp.set_bits;
  // 2. Thompson NFA; one MATCH per pattern
  std::vector<Inst> prog;
  std::vector<int> starts;
  for (size_t p = 0; p < pats.size(); p++) {
    NfaBuilder nb(*pats[p], prog, node_set[p], 400000);
    Frag f = nb.compile(pats[p]->root);
    Inst m;
    m.op = I_MATCH;
    m.arg = (int)p;
    int mpc = nb.emit(m);
    nb.patch(f.outs, mpc);
    if (nb.overflow) {
      *err = "regex too large";
      return false;
    }
    starts.push_back(f.start);
  }
  uint8_t used = 0;
  for (auto& in : prog)
    if (in.op == I_EMPTY) used |= in.assert_kind;
  const bool need_bol = used & (AS_BOT | AS_BOL);
  const bool need_word = used & (AS_WB | AS_NWB);

  // 3. subset construction (RE2-style flags, unanchored)
  enum { FL_BOT = 1, FL_NL = 2, FL_WORD = 4 };
  struct St {
    std::vector<int> kernel;
    uint8_t flags;
  };
  std::vector<St> states;
  std::unordered_map<std::string, uint32_t> smap;
  std::vector<uint32_t> mark(prog.size(), 0);
  uint32_t gen = 0;
  auto intern = [&](std::vector<int> k, uint8_t fl) -> uint32_t {
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    if (!need_bol) fl &= ~(FL_BOT | FL_NL);
    if (!need_word) fl &= ~FL_WORD;
    std::string key((const char*)k.data(), k.size() * sizeof(int));
    key.push_back((char)fl);
    auto it = smap.find(key);
    if (it != smap.end()) return it->second;
    uint32_t id = (uint32_t)states.size();
    states.push_back({std::move(k), fl});
    smap.emplace(std::move(key), id);
    return id;
  };
  const uint32_t ACCEPT = 0;
  if (!multi) {
    states.push_back({{}, 0});  // state 0 = absorbing ACCEPT
    smap.emplace(std::string("ACCEPT"), 0);
  }
  uint32_t start = intern(starts, FL_BOT);
  std::vector<int> stack;
  auto closure = [&](const std::vector<int>& kernel, uint8_t cond, std::vector<int>* cpcs) -> uint64_t {
    gen++;
    cpcs->clear();
    stack.assign(kernel.begin(), kernel.end());
    uint64_t matched = 0;
    while (!stack.empty()) {
      int pc = stack.back();
      stack.pop_back();
      if (pc < 0 || mark[pc] == gen) continue;
      mark[pc] = gen;
      const Inst& in = prog[pc];
      switch (in.op) {
        case I_MATCH: matched |= 1ull << in.arg; break;
        case I_CLASS: cpcs->push_back(pc); break;
        case I_NOP: stack.push_back(in.out); break;
        case I_SPLIT:
          stack.push_back(in.out1);
          stack.push_back(in.out);
          break;
        case I_EMPTY:
          if ((in.assert_kind & cond) == in.assert_kind) stack.push_back(in.out);
          break;
      }
    }
    return matched;
  };
  std::vector<uint16_t> trans;
  std::vector<uint8_t> end_acc;
  std::vector<uint64_t> acc;
  std::vector<int> nk;
  const uint32_t first = multi ? 0 : 1;
  const uint32_t id_cap = multi ? 0x7FFF : 0xFFFF;
  for (uint32_t sid = first; sid < states.size(); sid++) {
    if (states.size() > state_cap) {
      *err = "DFA exceeds state cap";
      return false;
    }
    const std::vector<int> kernel = states[sid].kernel;
    const uint8_t fl = states[sid].flags;
    trans.resize((size_t)(sid + 1) * ncls, 0);
    end_acc.resize(sid + 1, 0);
    if (multi) acc.resize((size_t)(sid + 1) * 5, 0);
    const bool bot = fl & FL_BOT, prevnl = fl & FL_NL, prevw = fl & FL_WORD;
    uint8_t base = 0;
    if (bot) base |= AS_BOT;
    if (bot || prevnl) base |= AS_BOL;
    {
      uint8_t cond = base | AS_EOT | AS_EOL | (prevw ? AS_WB : AS_NWB);
      std::vector<int> tmp;
      uint64_t m = closure(kernel, cond, &tmp);
      end_acc[sid] = m ? 1 : 0;
      if (multi) acc[(size_t)sid * 5 + 4] = m;
    }
    std::vector<int> cl[4];
    uint64_t clm[4] = {0, 0, 0, 0};
    bool have[4] = {false, false, false, false};
    for (uint32_t c = 0; c < ncls; c++) {
      const bool isnl = c == cls_nl, isw = cls_word[c];
      const int slot = (isnl ? 1 : 0) | (isw ? 2 : 0);
      if (!have[slot]) {
        uint8_t cond = base | (isnl ? AS_EOL : 0) | ((prevw != isw) ? AS_WB : AS_NWB);
        clm[slot] = closure(kernel, cond, &cl[slot]);
        have[slot] = true;
        if (multi) acc[(size_t)sid * 5 + slot] = clm[slot];
      }
      if (!multi && clm[slot]) {
        trans[(size_t)sid * ncls + c] = ACCEPT;
        continue;
      }
      nk.assign(starts.begin(), starts.end());
      for (int pc : cl[slot]) {
        const Inst& in = prog[pc];
        if (set_bits[in.arg][c >> 6] >> (c & 63) & 1) nk.push_back(in.out);
      }
      uint8_t nfl = (isnl ? FL_NL : 0) | (isw ? FL_WORD : 0);
      uint32_t t = intern(nk, nfl);
      if (t > id_cap) {
        *err = "DFA exceeds state cap";
        return false;
      }
      trans[(size_t)sid * ncls + c] = (uint16_t)(t | ((multi && clm[slot]) ? 0x8000 : 0));
    }
  }
  const uint32_t n = (uint32_t)states.size();
  trans.resize((size_t)n * ncls, 0);
  end_acc.resize(n, 0);
  if (!multi) {
    for (uint32_t c = 0; c < ncls; c++) trans[c] = ACCEPT;
    end_acc[0] = 1;
  } else {
    acc.resize((size_t)n * 5, 0);
  }
  out->n_states = n;
  out->start = start;
  out->accept = multi ? 0xFFFFFFFFu : ACCEPT;
  out->trans.swap(trans);
  out->end_accept.swap(end_acc);
  out->acc.swap(acc);
  minimize(out);
  if (multi) out->accept = 0xFFFF;  // no absorbing state
  return true;
}

}  // namespace

bool build_regex_dfa(const Regex& re, Dfa* out, std::string* err, uint32_t state_cap) {
  return build_core({&re}, false, out, err, state_cap);
}

bool build_union_dfa(const std::vector<const Regex*>& pats, Dfa* out, std::string* err, uint32_t state_cap,
                     uint32_t byte_budget) {
  return build_core(pats, true, out, err, state_cap, byte_budget);
}

// Position tables of the Thompson NFA (exact matcher for patterns whose DFA
// exceeds the state cap).  Positions = the NFA's class instructions.  The
// assertions between two runes depend only on what the previous and the next
// rune are (nothing / '\n' / word char / other), so the epsilon closure after
// a position is tabulated for those 16 combinations.
bool build_nfa_tables(const Regex& re, NfaTables* out, std::string* err, uint32_t max_pos) {
  *out = NfaTables();
  ClassPart cp;
  if (!partition_classes({&re}, &cp, err)) return false;
  std::vector<Inst> prog;
  NfaBuilder nb(re, prog, cp.node_set[0], 400000);
  Frag f = nb.compile(re.root);
  Inst m;
  m.op = I_MATCH;
  m.arg = 0;
  const int mpc = nb.emit(m);
  nb.patch(f.outs, mpc);
  if (nb.overflow) {
    *err = "regex too large";
    return false;
  }
  std::vector<int> pos_of(prog.size(), -1), pc_of;
  for (size_t pc = 0; pc < prog.size(); pc++)
    if (prog[pc].op == I_CLASS) {
      pos_of[pc] = (int)pc_of.size();
      pc_of.push_back((int)pc);
    }
  const uint32_t np = (uint32_t)pc_of.size();
  if (np > max_pos) {
    *err = "NFA exceeds position cap";
    return false;
  }
  const uint32_t W = (np + 1 + 63) / 64;  // + the match bit (bit np)
  out->n_classes = cp.ncls;
  out->n_pos = np;
  out->words = W;
  out->amap = cp.amap;
  out->nranges = cp.nranges;
  out->cls_combo = cp.cls_combo;
  out->cm.assign((size_t)cp.ncls * W, 0);
  for (uint32_t p = 0; p < np; p++) {
    const std::vector<uint64_t>& bits = cp.set_bits[prog[pc_of[p]].arg];
    for (uint32_t c = 0; c < cp.ncls; c++)
      if (bits[c >> 6] >> (c & 63) & 1) out->cm[(size_t)c * W + (p >> 6)] |= 1ull << (p & 63);
  }
  out->follow.assign((size_t)(np + 1) * 16 * W, 0);
  std::vector<uint32_t> mark(prog.size(), 0);
  uint32_t gen = 0;
  std::vector<int> stack;
  for (uint32_t row = 0; row <= np; row++) {
    for (uint32_t combo = 0; combo < 16; combo++) {
      const uint32_t prev = combo >> 2, next = combo & 3;  // 0 none, 1 '\n', 2 word, 3 other
      uint8_t cond = 0;
      if (prev == 0) cond |= AS_BOT | AS_BOL;
      if (prev == 1) cond |= AS_BOL;
      if (next == 0) cond |= AS_EOT | AS_EOL;
      if (next == 1) cond |= AS_EOL;
      cond |= ((prev == 2) != (next == 2)) ? AS_WB : AS_NWB;
      uint64_t* dst = &out->follow[((size_t)row * 16 + combo) * W];
      gen++;
      stack.clear();
      stack.push_back(row == np ? f.start : prog[pc_of[row]].out);
      while (!stack.empty()) {
        const int pc = stack.back();
        stack.pop_back();
        if (pc < 0 || mark[pc] == gen) continue;
        mark[pc] = gen;
        const Inst& in = prog[pc];
        switch (in.op) {
          case I_MATCH: dst[np >> 6] |= 1ull << (np & 63); break;
          case I_CLASS: dst[pos_of[pc] >> 6] |= 1ull << (pos_of[pc] & 63); break;
          case I_NOP: stack.push_back(in.out); break;
          case I_SPLIT:
            stack.push_back(in.out1);
            stack.push_back(in.out);
            break;
          case I_EMPTY:
            if ((in.assert_kind & cond) == in.assert_kind) stack.push_back(in.out);
            break;
        }
      }
    }
  }
  return true;
}

// Superset relaxations of a regex, for a phase-A prefilter automaton when the
// exact DFA exceeds the state cap: level 1 unbounds counted repetitions
// ({m,n} -> {m,}), level 2 also drops assertions (^ $ \b \B), level 3 also
// lowers repetition minima to 1.  Each step only removes constraints, so the
// relaxed language contains the original one.
void relax_regex(Regex* re, int level) {
  for (ReNode& n : re->nodes) {
    if (n.kind == N_REPEAT && n.max != -1 && n.max > n.min && level >= 1) n.max = -1;
    if (n.kind == N_REPEAT && level >= 3 && n.min > 1) {
      n.min = 1;
      n.max = -1;
    }
    if (n.kind == N_ASSERT && level >= 2) n.kind = N_EMPTY;
  }
}

// Host walk of the NFA tables (compiler self-test; the device runs the same
// algorithm in kernels.hip nfa_match).
bool nfa_host_match(const NfaTables& t, const uint8_t* s, size_t n) {
  const uint32_t W = t.words;
  std::vector<uint64_t> T(W, 0), S(W);
  uint32_t prev = 0;
  size_t i = 0;
  for (;;) {
    uint32_t cls = 0, next = 0;
    int w = 1;
    if (i < n) {
      const uint32_t r = s[i] < 0x80 ? s[i] : go_decode_rune(s, n, i, &w);
      if (r < 0x80) {
        cls = t.amap[r];
      } else {
        for (size_t k = 0; k + 2 < t.nranges.size(); k += 3)
          if (t.nranges[k] <= r && r <= t.nranges[k + 1]) cls = t.nranges[k + 2];
      }
      next = (t.cls_combo[cls] & 1) ? 1 : (t.cls_combo[cls] & 2) ? 2 : 3;
    }
    const uint32_t combo = prev * 4 + next;
    for (uint32_t k = 0; k < W; k++) S[k] = t.follow[((size_t)t.n_pos * 16 + combo) * W + k];
    for (uint32_t k = 0; k < W; k++)
      for (uint64_t b = T[k]; b; b &= b - 1) {
        const uint32_t p = k * 64 + __builtin_ctzll(b);
        for (uint32_t j = 0; j < W; j++) S[j] |= t.follow[((size_t)p * 16 + combo) * W + j];
      }
    if (S[t.n_pos >> 6] >> (t.n_pos & 63) & 1) return true;
    if (i >= n) return false;
    for (uint32_t k = 0; k < W; k++) T[k] = S[k] & t.cm[(size_t)cls * W + k];
    prev = next;
    i += w;
  }
}

bool phrases_to_regex(const std::vector<std::string>& phrases, bool fold_ascii, Regex* out) {
  *out = Regex();
  std::vector<int> alts;
  for (auto& p : phrases) {
    std::vector<int> lits;
    for (uint8_t c : p) {
      if (c >= 0x80) return false;
      ReNode n;
      n.kind = N_CLASS;
      if (fold_ascii && c >= 'a' && c <= 'z') n.set = {{(uint32_t)c - 32, (uint32_t)c - 32}, {c, c}};
      else if (fold_ascii && c >= 'A' && c <= 'Z') n.set = {{c, c}, {(uint32_t)c + 32, (uint32_t)c + 32}};
      else n.set = {{c, c}};
      out->nodes.push_back(n);
      lits.push_back((int)out->nodes.size() - 1);
    }
    ReNode cat;
    if (lits.empty()) {
      cat.kind = N_EMPTY;
    } else {
      cat.kind = N_CAT;
      cat.kids = lits;
    }
    out->nodes.push_back(cat);
    alts.push_back((int)out->nodes.size() - 1);
  }
  if (alts.empty()) {
    // no phrase: never matches -> empty class
    ReNode n;
    n.kind = N_CLASS;
    out->nodes.push_back(n);
    out->root = (int)out->nodes.size() - 1;
    return true;
  }
  ReNode alt;
  alt.kind = N_ALT;
  alt.kids = alts;
  out->nodes.push_back(alt);
  out->root = (int)out->nodes.size() - 1;
  return true;
}

// Aho-Corasick phrase automaton as a sticky byte DFA.
bool build_phrase_dfa(const std::vector<std::string>& phrases, bool fold_ascii, Dfa* out, std::string* err,
                      uint32_t state_cap) {
  *out = Dfa();
  out->byte_mode = true;
  auto fb = [&](uint8_t c) -> uint8_t { return (fold_ascii && c >= 'A' && c <= 'Z') ? c + 32 : c; };
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
  std::queue<int> q;
  for (uint32_t k = 0; k < ncls; k++) {
    int c = t[0].next[k];
    if (c < 0) {
      t[0].next[k] = 0;
    } else {
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

static uint32_t host_class(const Dfa& d, const uint8_t* s, size_t n, size_t* i) {
  if (d.byte_mode || s[*i] < 0x80) return d.amap[s[(*i)++]];
  int w;
  uint32_t r = go_decode_rune(s, n, *i, &w);
  *i += w;
  for (size_t k = 0; k + 2 < d.nranges.size(); k += 3)
    if (r >= d.nranges[k] && r <= d.nranges[k + 1]) return d.nranges[k + 2];
  return 0;
}

bool dfa_host_match(const Dfa& d, const uint8_t* s, size_t n) {
  if (d.multi) {
    uint64_t m = 0;
    uint32_t st = d.start;
    size_t i = 0;
    while (i < n) {
      uint32_t c = host_class(d, s, n, &i);
      uint16_t t = d.trans[(size_t)st * d.n_classes + c];
      if (t & 0x8000) m |= d.acc[(size_t)st * 5 + d.cls_combo[c]];
      st = t & 0x7FFF;
    }
    m |= d.acc[(size_t)st * 5 + 4];
    return m != 0;
  }
  uint32_t st = d.start;
  size_t i = 0;
  while (i < n) {
    if (st == d.accept) return true;
    uint32_t c = host_class(d, s, n, &i);
    st = d.trans[(size_t)st * d.n_classes + c];
  }
  return d.end_accept[st] != 0;
}

uint64_t dfa_host_scan(const Dfa& d, const uint8_t* s, size_t n) {
  if (!d.multi) return dfa_host_match(d, s, n) ? 1 : 0;
  uint64_t m = 0;
  uint32_t st = d.start;
  size_t i = 0;
  while (i < n) {
    uint32_t c = host_class(d, s, n, &i);
    uint16_t t = d.trans[(size_t)st * d.n_classes + c];
    if (t & 0x8000) m |= d.acc[(size_t)st * 5 + d.cls_combo[c]];
    st = t & 0x7FFF;
  }
  return m | d.acc[(size_t)st * 5 + 4];
}

}  // namespace gi
