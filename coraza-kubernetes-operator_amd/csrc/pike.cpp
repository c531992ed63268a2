// Regex AST -> Pike VM program (pike.h) for `capture` submatch extraction.
//
// Restates how Go compiles a parsed regexp for its NFA matcher
// [upstream Go regexp/syntax/simplify.go (counted repetition expansion) and
// compile.go (Alt / Quest / Star / Plus priorities, Capture slots)]:
//   * x|y      Alt(x, y): x preferred
//   * x?  x??  Alt(x, skip) / Alt(skip, x)
//   * x*  x*?  loop; a nullable x compiles as (x+)? (golang.org/issue/46123)
//   * x+  x+?  x then Alt(back to x, out) / Alt(out, back to x)
//   * x{n,m}   n copies of x, then (x(x(x)?)?)? with the same greediness;
//              x{n,} = n-1 copies then x+; x{0} matches empty
//   * (x)      Save(2k) x Save(2k+1); group 0 is set by the VM itself
// Used only for `capture` links whose TX.0-TX.8 values are observable
// (compile.cpp capture analysis).
#include <stdint.h>

#include <string>
#include <vector>

#include "pike.h"
#include "regex.h"

namespace gi {
namespace {

struct PFrag {
  uint32_t start;
  std::vector<std::pair<uint32_t, int>> outs;  // (inst, 0 = x / 1 = y) to patch
  bool nullable;
};

struct PikeBuilder {
  const Regex& re;
  std::vector<DPikeInst>& prog;
  std::vector<uint32_t>& pool;
  uint32_t max_inst;
  uint32_t nslot;
  bool overflow = false;

  uint32_t emit(uint8_t op, uint8_t aux = 0) {
    if (prog.size() >= max_inst) overflow = true;
    DPikeInst I{};
    I.op = op;
    I.aux = aux;
    I.x = I.y = 0;
    prog.push_back(I);
    return (uint32_t)prog.size() - 1;
  }
  void patch(const std::vector<std::pair<uint32_t, int>>& outs, uint32_t to) {
    for (auto& o : outs) (o.second ? prog[o.first].y : prog[o.first].x) = to;
  }
  PFrag nop() {
    uint32_t k = emit(PK_JMP);
    return {k, {{k, 0}}, true};
  }
  PFrag cat(PFrag a, PFrag b) {
    patch(a.outs, b.start);
    return {a.start, std::move(b.outs), a.nullable && b.nullable};
  }
  PFrag quest(PFrag x, bool greedy) {
    uint32_t s = emit(PK_SPLIT);
    if (greedy) {
      prog[s].x = x.start;
      x.outs.push_back({s, 1});
    } else {
      prog[s].y = x.start;
      x.outs.push_back({s, 0});
    }
    return {s, std::move(x.outs), true};
  }
  // loop: L: Split(x, out) ; x -> L
  PFrag loop(PFrag x, bool greedy) {
    uint32_t s = emit(PK_SPLIT);
    std::vector<std::pair<uint32_t, int>> outs;
    if (greedy) {
      prog[s].x = x.start;
      outs.push_back({s, 1});
    } else {
      prog[s].y = x.start;
      outs.push_back({s, 0});
    }
    patch(x.outs, s);
    return {s, std::move(outs), true};
  }
  PFrag star(PFrag x, bool greedy) {
    if (x.nullable) return quest(plus(std::move(x), greedy), greedy);
    return loop(std::move(x), greedy);
  }
  PFrag plus(PFrag x, bool greedy) {
    const uint32_t st = x.start;
    const bool nl = x.nullable;
    PFrag l = loop(std::move(x), greedy);
    return {st, std::move(l.outs), nl};
  }
  PFrag cls(const RuneSet& set) {
    uint32_t k = emit(PK_RUNE);
    DPikeInst& I = prog[k];
    I.roff = (uint32_t)pool.size();
    for (const RuneRange& r : set) {
      for (uint32_t c = r.lo; c <= r.hi && c < 128; c++) I.ascii[c >> 5] |= 1u << (c & 31);
      if (r.hi >= 128) {
        pool.push_back(r.lo < 128 ? 128u : r.lo);
        pool.push_back(r.hi);
      }
    }
    I.rcnt = (uint32_t)(pool.size() - I.roff) / 2;
    return {k, {{k, 0}}, false};
  }
  PFrag compile(int id) {
    if (overflow) return nop();
    const ReNode& n = re.nodes[id];
    switch (n.kind) {
      case N_CLASS:
        return cls(n.set);
      case N_EMPTY:
        return nop();
      case N_ASSERT: {
        uint8_t m = 0;
        if (n.assert_kind & AS_BOT) m |= PKE_BEGIN_TEXT;
        if (n.assert_kind & AS_EOT) m |= PKE_END_TEXT;
        if (n.assert_kind & AS_BOL) m |= PKE_BEGIN_LINE;
        if (n.assert_kind & AS_EOL) m |= PKE_END_LINE;
        if (n.assert_kind & AS_WB) m |= PKE_WORD_BOUNDARY;
        if (n.assert_kind & AS_NWB) m |= PKE_NO_WORD_BOUNDARY;
        uint32_t k = emit(PK_ASSERT, m);
        return {k, {{k, 0}}, true};
      }
      case N_CAPTURE: {
        const uint32_t s0 = emit(PK_SAVE, (uint8_t)std::min<uint32_t>(2u * n.cap, 255u));
        PFrag body = compile(n.kids[0]);
        const uint32_t s1 = emit(PK_SAVE, (uint8_t)std::min<uint32_t>(2u * n.cap + 1, 255u));
        prog[s0].x = body.start;
        patch(body.outs, s1);
        return {s0, {{s1, 0}}, body.nullable};
      }
      case N_CAT: {
        PFrag f = compile(n.kids[0]);
        for (size_t k = 1; k < n.kids.size(); k++) f = cat(std::move(f), compile(n.kids[k]));
        return f;
      }
      case N_ALT: {
        PFrag f = compile(n.kids.back());
        for (int k = (int)n.kids.size() - 2; k >= 0; k--) {
          PFrag a = compile(n.kids[k]);
          uint32_t s = emit(PK_SPLIT);
          prog[s].x = a.start;
          prog[s].y = f.start;
          std::vector<std::pair<uint32_t, int>> outs = std::move(a.outs);
          outs.insert(outs.end(), f.outs.begin(), f.outs.end());
          f = {s, std::move(outs), a.nullable || f.nullable};
        }
        return f;
      }
      case N_REPEAT: {
        const int sub = n.kids[0];
        const bool g = n.greedy;
        if (n.min == 0 && n.max == 0) return nop();
        if (n.max == -1) {
          if (n.min == 0) return star(compile(sub), g);
          if (n.min == 1) return plus(compile(sub), g);
          PFrag f = compile(sub);
          for (int k = 1; k < n.min - 1; k++) f = cat(std::move(f), compile(sub));
          return cat(std::move(f), plus(compile(sub), g));
        }
        if (n.min == 1 && n.max == 1) return compile(sub);
        PFrag f;
        bool have = false;
        for (int k = 0; k < n.min; k++) {
          PFrag c = compile(sub);
          f = have ? cat(std::move(f), std::move(c)) : std::move(c);
          have = true;
        }
        if (n.max > n.min) {
          PFrag suf = quest(compile(sub), g);
          for (int k = n.min + 1; k < n.max; k++) {
            PFrag c = compile(sub);
            suf = quest(cat(std::move(c), std::move(suf)), g);
          }
          f = have ? cat(std::move(f), std::move(suf)) : std::move(suf);
        }
        return f;
      }
    }
    return nop();
  }
};

}  // namespace

bool build_pike(const Regex& re, std::vector<DPikeInst>* insts, std::vector<uint32_t>* pool, DPike* out,
                std::string* err, uint32_t max_inst) {
  const uint32_t base = (uint32_t)insts->size();
  std::vector<DPikeInst> prog;
  std::vector<uint32_t> rp;
  PikeBuilder b{re, prog, rp, max_inst, 0};
  PFrag f = b.compile(re.root);
  const uint32_t m = b.emit(PK_MATCH);
  b.patch(f.outs, m);
  if (b.overflow) {
    *err = "capture program over " + std::to_string(max_inst) + " instructions";
    return false;
  }
  // relocate into the shared arrays
  const uint32_t roff = (uint32_t)pool->size();
  for (DPikeInst& I : prog)  // x / y stay relative to the program (the VM indexes prog + inst_off)
    if (I.op == PK_RUNE) I.roff += roff;
  insts->insert(insts->end(), prog.begin(), prog.end());
  pool->insert(pool->end(), rp.begin(), rp.end());
  out->inst_off = base;
  out->n_inst = (uint32_t)prog.size();
  out->start = f.start;  // relative to inst_off
  out->nslot = 2u * (uint32_t)std::min(re.ncap + 1, 9);
  return true;
}

}  // namespace gi
