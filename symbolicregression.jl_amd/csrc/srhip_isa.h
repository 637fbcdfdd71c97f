// srhip_isa.h — the device bytecode ("postfix accumulator/stack machine") shared by the host
// compiler (srhip_compile.cpp) and the gfx950 interpreter (srhip_eval_impl.h).
//
// Machine model (one wavefront, R rows per lane, all state in VGPRs):
//   A      accumulator: the value of the subexpression being evaluated (R values per lane)
//   S[k]   stack slots k < K (Sethi-Ullman ordering keeps K = Strahler number - 1 small)
//   X[f]   feature f of the current row tile, read from LDS
// Every operator instruction also folds max|A| (NaN-propagating) into the tree's check
// accumulator: that is the device side of DynamicExpressions' did_succeed checks (see
// DESIGN.md "did_succeed"). Instruction = 16 bytes, read with one s_load_dwordx4 (wave-uniform).
#pragma once
#include <stdint.h>

#include "../../include/srhip.h"

namespace srhip {

constexpr int K_MAX = 8;  // stack slots in the largest kernel variant

// Binary operators specialised for every operand form (cheap or very common).
#define SRHIP_SPEC_BINOPS(X)                                                                \
  X(ADD, add) X(SUB, sub) X(MUL, mul) X(DIV, div) X(GREATER, greater) X(COND, cond)           \
  X(LOGICAL_OR, logical_or) X(LOGICAL_AND, logical_and) X(MAX, max) X(MIN, min)
// Binary operators with large bodies (out of line): A = S[k] op A or A = A op S[k].
#define SRHIP_HEAVY_BINOPS(X) X(POW, pow) X(MOD, mod) X(ATAN2, atan2)
#define SRHIP_UNOPS(X)                                                                         \
  X(NEG, neg) X(SQUARE, square) X(CUBE, cube) X(ABS, abs) X(RELU, relu) X(COS, cos) X(SIN, sin) \
  X(TAN, tan) X(EXP, exp) X(LOG, log) X(LOG2, log2) X(LOG10, log10) X(LOG1P, log1p)            \
  X(SQRT, sqrt) X(ACOSH, acosh) X(ATANH_CLIP, atanh_clip) X(SINH, sinh) X(COSH, cosh)          \
  X(TANH, tanh) X(ASIN, asin) X(ACOS, acos) X(ATAN, atan) X(ASINH, asinh) X(ERF, erf)          \
  X(ERFC, erfc) X(GAMMA, gamma) X(ROUND, round) X(FLOOR, floor) X(CEIL, ceil) X(SIGN, sign)    \
  X(EXP2, exp2) X(EXPM1, expm1) X(CBRT, cbrt)

enum SpecBin : int {
#define X_(n, f) SB_##n,
  SRHIP_SPEC_BINOPS(X_)
#undef X_
  NUM_SPEC_BIN
};
enum HeavyBin : int {
#define X_(n, f) HB_##n,
  SRHIP_HEAVY_BINOPS(X_)
#undef X_
  NUM_HEAVY_BIN
};
enum Unop : int {
#define X_(n, f) UN_##n,
  SRHIP_UNOPS(X_)
#undef X_
  NUM_UNOP
};

// Unary operators cheap enough to inline into their handler (a few VALU instructions per row).
constexpr bool un_cheap(int u) {
  return u == UN_NEG || u == UN_SQUARE || u == UN_CUBE || u == UN_ABS || u == UN_RELU || u == UN_SIGN ||
         u == UN_ROUND || u == UN_FLOOR || u == UN_CEIL;
}
// "Wide" unary operators (OCML bodies with ~100 live VGPRs): only the K = K_MAX variant has them.
constexpr bool un_wide_op(int u) { return u == UN_ASIN || u == UN_ACOS || u == UN_ATANH_CLIP; }

// Derived columns: a heavy unary operator applied directly to a feature leaf, U(X[f]), has the same
// value in every tree of a population.  The host lists the (U, f) pairs a program uses at least
// DERIVE_MIN_USES times; each workgroup computes them once for its rows into LDS columns after the
// staged features (same out-of-line operator bodies, so bit-identical values) and the trees read
// them like features.  A derived column d is LDS column (staged features + d).
constexpr int DERIVE_MAX = 16;
constexpr int DERIVE_MIN_USES = 2;
constexpr bool un_derivable(int u) { return u >= 0 && !un_cheap(u) && !un_wide_op(u); }

// ---- handler ids -----------------------------------------------------------------------------
enum : uint32_t {
  H_END = 0,
  H_LOADF = 1,                        // A = X[a]
  H_LOADC = 2,                        // A = imm
  H_SLOADF0 = 3,                      // S[k] = X[a]   (operand of a heavy binary op)
  H_SLOADC0 = H_SLOADF0 + K_MAX,      // S[k] = imm
  H_PUSH0 = H_SLOADC0 + K_MAX,        // S[k] = A
  // superinstructions (evaluation programs; gradient programs as SRHIP_GRAD_SUPER_LEVEL below allows):
  H_PUSHLF0 = H_PUSH0 + K_MAX,        // S[k] = A; A = X[a]     (a push followed by a feature leaf)
  H_PUSHLC0 = H_PUSHLF0 + K_MAX,      // S[k] = A; A = imm      (a push followed by a constant leaf)
  H_BIN0 = H_PUSHLC0 + K_MAX,         // specialised binary ops, SPEC_STRIDE handlers each
};
// operand forms of a specialised binary op: A op X[a], X[a] op A, A op imm, imm op A, S[k] op A,
// A op S[k], and the leaf-leaf forms of DynamicExpressions' deg2_l0_r0 (one instruction instead of a
// load and an op): X[a] op X[imm], X[a] op imm, imm op X[a]
constexpr uint32_t SPEC_AF = 0, SPEC_FA = 1, SPEC_AC = 2, SPEC_CA = 3, SPEC_SA0 = 4,
                   SPEC_AS0 = 4 + K_MAX, SPEC_FF = 4 + 2 * K_MAX, SPEC_FC = SPEC_FF + 1, SPEC_CF = SPEC_FF + 2,
                   SPEC_STRIDE = SPEC_FF + 3;
// the superinstructions a gradient program uses (and the gradient kernel implements; srhip_grad.hip):
// 0 none, 1 the push-load pairs (H_PUSHLF0 / H_PUSHLC0), 2 those and the leaf-leaf forms (SPEC_FF /
// SPEC_FC / SPEC_CF, the constant's index in the operand's upper half).  Exact at every level; 0 by
// default: C4 measured 146.2 / 149.2 / 146.3 ms per step at level 0, 146.6 / 149.7 / 146.1 at 1 and
// 149.1 / 148.9 / 145.9 at 2 (same box, interleaved), and the gradient kernel's roofline fraction fell
// 0.0368 -> 0.0350 with the handlers in: a quarter fewer dispatches, each in a larger kernel (every
// variant grows; they run concurrently from several streams and share the instruction cache).
#ifndef SRHIP_GRAD_SUPER_LEVEL
#define SRHIP_GRAD_SUPER_LEVEL 0
#endif
// heavy binary ops take their second operand from a stack slot: A = S[k] op A, or A = A op S[k]
constexpr uint32_t HEAVY_SA0 = 0, HEAVY_AS0 = K_MAX, HEAVY_STRIDE = 2 * K_MAX;
constexpr uint32_t H_HEAVY0 = H_BIN0 + NUM_SPEC_BIN * SPEC_STRIDE;
constexpr uint32_t H_UN0 = H_HEAVY0 + NUM_HEAVY_BIN * HEAVY_STRIDE;
constexpr uint32_t H_COUNT = H_UN0 + NUM_UNOP;
// operand flag of a cos / sin instruction whose operand is an operator output: no check fold of its
// own -- |cos|, |sin| <= 1, and a non-finite result needs a non-finite operand, which the operand's
// own instruction folded (the host sets it only for that case; a feature-leaf operand keeps the
// checked form).  A flag, not a handler of its own: one call site per operator in the interpreter
// (round 5: the separate handlers' call site carried a 64-byte register spill on its dispatch path)
constexpr uint32_t UN_NC_FLAG = 0x8000;
// operand flag of a gradient-program unary instruction whose operand is a constant subtree: the
// operand's rows all hold one value (and one tangent), so the kernel evaluates the operator on one row
// and copies it to the others -- the same bits, one evaluation per lane instead of R
constexpr uint32_t UN_UNIFORM_FLAG = 0x4000;
// unary operators the gradient kernel evaluates inline (a few instructions, exact derivative); the rest
// are "heavy" calls -- those a gradient program reads from derived columns when applied to a feature
constexpr bool un_grad_inline(int u) {
  return u == UN_NEG || u == UN_SQUARE || u == UN_CUBE || u == UN_ABS || u == UN_RELU || u == UN_SIGN ||
         u == UN_ROUND || u == UN_FLOOR || u == UN_CEIL;
}

constexpr uint32_t h_spec(int sb, uint32_t form) { return H_BIN0 + uint32_t(sb) * SPEC_STRIDE + form; }
constexpr uint32_t h_heavy(int hb, uint32_t form) { return H_HEAVY0 + uint32_t(hb) * HEAVY_STRIDE + form; }
constexpr uint32_t h_un(int u) { return H_UN0 + uint32_t(u); }

struct __attribute__((aligned(16))) Ins {
  uint32_t h;    // handler id
  uint32_t a;    // feature index (0-based) or stack slot
  uint64_t imm;  // constant bits: f32/i32 in the low word, f64 full
};
static_assert(sizeof(Ins) == 16, "Ins must be 16 bytes");

// Map public SRHIP_OP_* codes to the internal categories; returns false if unknown.
inline bool classify_binop(int code, int* spec, int* heavy) {
  *spec = -1;
  *heavy = -1;
  switch (code) {
#define X_(n, f) \
  case SRHIP_OP_##n: *spec = SB_##n; return true;
    SRHIP_SPEC_BINOPS(X_)
#undef X_
#define X_(n, f) \
  case SRHIP_OP_##n: *heavy = HB_##n; return true;
    SRHIP_HEAVY_BINOPS(X_)
#undef X_
    default: return false;
  }
}
inline int classify_unop(int code) {
  switch (code) {
#define X_(n, f) \
  case SRHIP_OP_##n: return UN_##n;
    SRHIP_UNOPS(X_)
#undef X_
    default: return -1;
  }
}

// Integer-typed trees (Node{Int32}) support only wrap-around ring ops and comparisons
// (Julia Int32 semantics; `/` on Int32 returns Float64 in Julia and is rejected).
inline bool int_binop_ok(int code) {
  switch (code) {
    case SRHIP_OP_ADD: case SRHIP_OP_SUB: case SRHIP_OP_MUL: case SRHIP_OP_GREATER:
    case SRHIP_OP_COND: case SRHIP_OP_LOGICAL_OR: case SRHIP_OP_LOGICAL_AND:
    case SRHIP_OP_MAX: case SRHIP_OP_MIN:
      return true;
    default: return false;
  }
}
inline bool int_unop_ok(int code) {
  switch (code) {
    case SRHIP_OP_NEG: case SRHIP_OP_SQUARE: case SRHIP_OP_CUBE: case SRHIP_OP_ABS:
    case SRHIP_OP_RELU: case SRHIP_OP_SIGN:
      return true;
    default: return false;
  }
}

}  // namespace srhip
