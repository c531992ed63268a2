// Submatch extraction for `capture` (TX.0-TX.8): a Pike VM with Go regexp's
// leftmost-first priorities.
//
// [upstream coraza/v3 v3.3.3 internal/operators/rx.go]: with capturing on,
// @rx calls regexp.FindStringSubmatch and writes group i to TX.i for i < 9.
// Go's regexp answers FindStringSubmatch with its one-pass, backtracking or
// NFA ("pike") matcher -- all three give the leftmost-first match.  This
// header restates the NFA one (regexp/exec.go machine.match / step / add over
// a syntax.Prog compiled like regexp/syntax/compile.go): threads are kept in
// priority order, a Match cuts every lower-priority thread, and new threads
// start at each position only until a match is found.
//
// The same function runs in k_eval (device) and in the compiler self-test
// (host: gi_selftest_capture), so the CPU tests pin the VM against the oracle.
#pragma once
#include <stdint.h>

#if !defined(__HIPCC__) && !defined(__host__)
#define __host__
#define __device__
#endif

namespace gi {

enum PikeOp : uint8_t { PK_RUNE = 1, PK_SPLIT, PK_JMP, PK_SAVE, PK_ASSERT, PK_MATCH, PK_FAIL };

// One instruction (36 B).  PK_SPLIT: x preferred over y; PK_JMP / PK_SAVE /
// PK_ASSERT / PK_RUNE continue at x.  PK_SAVE: aux = capture slot (2 g start,
// 2 g + 1 end).  PK_ASSERT: aux = the empty-width ops that must hold (PKE_*).
// PK_RUNE: ASCII bitmap + sorted (lo, hi) pairs for runes >= 0x80 in the u32
// pool at roff.
struct DPikeInst {
  uint8_t op, aux;
  uint16_t _pad;
  uint32_t x, y;
  uint32_t roff, rcnt;
  uint32_t ascii[4];
};

struct DPike {
  uint32_t inst_off, n_inst;
  uint32_t nslot;  // capture slots tracked: 2 x (groups + 1), at most 18 (TX.0-TX.8)
  uint32_t start;
  uint32_t whole;  // the pattern is (?sm)^.*$: every value matches whole (group 0 = [0, n)), no VM run
};

// Go regexp/syntax EmptyOp bits
enum : uint32_t {
  PKE_BEGIN_LINE = 1, PKE_END_LINE = 2, PKE_BEGIN_TEXT = 4, PKE_END_TEXT = 8,
  PKE_WORD_BOUNDARY = 16, PKE_NO_WORD_BOUNDARY = 32,
};

#define GI_PIKE_MAX_SLOTS 18

// Workspace words pike_match needs for a program of n_inst instructions.
__host__ __device__ inline uint64_t pike_ws_words(uint32_t n_inst, uint32_t nslot) {
  // two thread queues (pc + slots per entry) + two generation-stamp arrays +
  // the add() stack (at most 3 entries of 2 words per instruction) + counters
  return 2ull * n_inst * (1 + nslot) + 2ull * n_inst + 6ull * n_inst + 8;
}

__host__ __device__ inline bool pike_word(int32_t r) {
  return r == '_' || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || (r >= '0' && r <= '9');
}

// syntax.EmptyOpContext(r1, r2): r1 the rune before the position, r2 after (-1: text edge)
__host__ __device__ inline uint32_t pike_context(int32_t r1, int32_t r2) {
  uint32_t op = PKE_NO_WORD_BOUNDARY;
  uint32_t boundary = 0;
  if (pike_word(r1)) boundary = 1;
  else if (r1 == '\n') op |= PKE_BEGIN_LINE;
  else if (r1 < 0) op |= PKE_BEGIN_TEXT | PKE_BEGIN_LINE;
  if (pike_word(r2)) boundary ^= 1;
  else if (r2 == '\n') op |= PKE_END_LINE;
  else if (r2 < 0) op |= PKE_END_TEXT | PKE_END_LINE;
  if (boundary) op ^= (PKE_WORD_BOUNDARY | PKE_NO_WORD_BOUNDARY);
  return op;
}

// utf8.DecodeRune at s[i] (i < n): invalid -> U+FFFD, width 1
__host__ __device__ inline int32_t pike_decode(const uint8_t* s, uint32_t n, uint32_t i, uint32_t* w) {
  const uint8_t c0 = s[i];
  *w = 1;
  if (c0 < 0x80) return c0;
  uint32_t need;
  uint8_t lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) need = 1;
  else if (c0 == 0xE0) { need = 2; lo = 0xA0; }
  else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) need = 2;
  else if (c0 == 0xED) { need = 2; hi = 0x9F; }
  else if (c0 == 0xF0) { need = 3; lo = 0x90; }
  else if (c0 >= 0xF1 && c0 <= 0xF3) need = 3;
  else if (c0 == 0xF4) { need = 3; hi = 0x8F; }
  else return 0xFFFD;
  if (n - i < need + 1) return 0xFFFD;
  const uint8_t c1 = s[i + 1];
  if (c1 < lo || c1 > hi) return 0xFFFD;
  for (uint32_t k = 2; k <= need; k++)
    if (s[i + k] < 0x80 || s[i + k] > 0xBF) return 0xFFFD;
  *w = need + 1;
  if (need == 1) return ((c0 & 0x1F) << 6) | (c1 & 0x3F);
  if (need == 2) return ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (s[i + 2] & 0x3F);
  return ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
}

__host__ __device__ inline bool pike_rune_in(const DPikeInst& I, const uint32_t* rpool, int32_t r) {
  if (r < 0) return false;
  if (r < 128) return (I.ascii[r >> 5] >> (r & 31)) & 1u;
  uint32_t lo = 0, hi = I.rcnt;
  const uint32_t* rr = rpool + I.roff;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (rr[2 * mid + 1] < (uint32_t)r) lo = mid + 1;
    else hi = mid;
  }
  return lo < I.rcnt && rr[2 * lo] <= (uint32_t)r;
}

// FindStringSubmatch over s[0, n): true on a match, caps[0 .. pk.nslot) =
// byte offsets (-1: the group did not participate).  ws: pike_ws_words words.
// Work is bounded by (n + 1) x n_inst steps (no backtracking).
__host__ __device__ inline bool pike_match(const DPikeInst* prog, const uint32_t* rpool, const DPike& pk,
                                           const uint8_t* s, uint32_t n, uint32_t* ws, int32_t* caps) {
  const uint32_t NI = pk.n_inst, NS = pk.nslot, TW = 1 + NS;
  uint32_t* qd[2] = {ws, ws + (uint64_t)NI * TW};          // thread entries: pc, slots
  uint32_t* qm[2] = {ws + 2ull * NI * TW, ws + 2ull * NI * TW + NI};  // generation stamps per pc
  uint32_t* stk = ws + 2ull * NI * TW + 2ull * NI;       // (word0, word1) entries
  uint32_t qn[2] = {0, 0};
  uint32_t gen[2] = {1, 2};
  for (uint32_t k = 0; k < 2 * NI; k++) qm[0][k] = 0;
  int32_t cap[GI_PIKE_MAX_SLOTS], mcap[GI_PIKE_MAX_SLOTS];
  for (uint32_t k = 0; k < NS; k++) mcap[k] = -1;
  bool matched = false;
  // add(q, pc, pos, cap, ctx): the epsilon closure in priority order (regexp/exec.go add)
  auto add = [&](uint32_t q, uint32_t pc0, uint32_t pos, uint32_t ctx) {
    // stack entries: (pc, 0) to explore, (0x80000000 | slot, old value) to restore
    uint32_t sp = 0;
    stk[0] = pc0;
    stk[1] = 0;
    sp = 1;
    while (sp) {
      sp--;
      const uint32_t a = stk[2 * sp], b = stk[2 * sp + 1];
      if (a & 0x80000000u) {
        cap[a & 0x7FFFFFFFu] = (int32_t)b;
        continue;
      }
      const uint32_t pc = a;
      if (qm[q][pc] == gen[q]) continue;
      qm[q][pc] = gen[q];
      const DPikeInst& I = prog[pc];
      switch (I.op) {
        case PK_SPLIT:
          stk[2 * sp] = I.y, stk[2 * sp + 1] = 0, sp++;
          stk[2 * sp] = I.x, stk[2 * sp + 1] = 0, sp++;
          break;
        case PK_JMP:
          stk[2 * sp] = I.x, stk[2 * sp + 1] = 0, sp++;
          break;
        case PK_ASSERT:
          if ((I.aux & ~ctx) == 0) stk[2 * sp] = I.x, stk[2 * sp + 1] = 0, sp++;
          break;
        case PK_SAVE:
          if (I.aux < NS) {
            stk[2 * sp] = 0x80000000u | I.aux, stk[2 * sp + 1] = (uint32_t)cap[I.aux], sp++;
            cap[I.aux] = (int32_t)pos;
          }
          stk[2 * sp] = I.x, stk[2 * sp + 1] = 0, sp++;
          break;
        case PK_RUNE:
        case PK_MATCH: {
          uint32_t* t = qd[q] + (uint64_t)qn[q] * TW;
          t[0] = pc;
          for (uint32_t k = 0; k < NS; k++) t[1 + k] = (uint32_t)cap[k];
          qn[q]++;
          break;
        }
        default:
          break;  // PK_FAIL
      }
    }
  };
  uint32_t w = 0, w1 = 0;
  int32_t r = n ? pike_decode(s, n, 0, &w) : -1;
  int32_t r1 = -1;
  if (r >= 0 && w < n) r1 = pike_decode(s, n, w, &w1);
  uint32_t ctx = pike_context(-1, r);
  uint32_t pos = 0, cur = 0;
  for (;;) {
    if (qn[cur] == 0 && matched) break;
    if (!matched) {
      for (uint32_t k = 0; k < NS; k++) cap[k] = -1;
      if (NS) cap[0] = (int32_t)pos;
      add(cur, pk.start, pos, ctx);
    }
    const uint32_t nctx = pike_context(r, r1);
    const uint32_t nxt = cur ^ 1u;
    // step: the threads of cur in priority order
    for (uint32_t j = 0; j < qn[cur]; j++) {
      const uint32_t* t = qd[cur] + (uint64_t)j * TW;
      const DPikeInst& I = prog[t[0]];
      if (I.op == PK_MATCH) {
        for (uint32_t k = 0; k < NS; k++) mcap[k] = (int32_t)t[1 + k];
        if (NS > 1) mcap[1] = (int32_t)pos;
        matched = true;
        break;  // first-match mode: lower-priority threads are cut
      }
      if (w > 0 && pike_rune_in(I, rpool, r)) {
        for (uint32_t k = 0; k < NS; k++) cap[k] = (int32_t)t[1 + k];
        add(nxt, I.x, pos + w, nctx);
      }
    }
    qn[cur] = 0;
    gen[cur] += 2;
    if (w == 0) break;
    pos += w;
    r = r1;
    w = w1;
    r1 = -1;
    w1 = 0;
    if (r >= 0 && pos + w < n) r1 = pike_decode(s, n, pos + w, &w1);
    ctx = nctx;
    cur = nxt;
  }
  for (uint32_t k = 0; k < NS; k++) caps[k] = mcap[k];
  return matched;
}

}  // namespace gi
