// srhip_grad.h — argument block and launchers of the constant-gradient kernels (srhip_grad.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srhip_isa.h"

namespace srhip {

constexpr int GRAD_WAVES = 8;  // wavefronts per workgroup
constexpr int GRAD_KT = 8;     // tangent components per pass (constants per chunk)
// What a launch computes:
//   GMODE_LOSS  loss + d loss / d constants per (chunk, row block) -> slab (the optimiser's objective)
//   GMODE_ROWC  per-row d out / d constants -> out_der (eval_grad_tree_array, variable = false)
//   GMODE_ROWF  per-row d out / d features -> out_der (variable = true, and eval_diff_tree_array)
constexpr int GMODE_LOSS = 0, GMODE_ROWC = 1, GMODE_ROWF = 2;
constexpr int GRAD_ROW_KT = 4;  // tangent components per chunk of the per-row modes

struct GradArgs {
  const Ins* code;          // gradient programs of all trees
  const int32_t* prog_off;  // [ntrees]
  const int32_t* chunks;    // GMODE_LOSS: [nchunks][2] (tree, first constant); per-row modes:
                            // [nchunks][4] (tree, first component c0, end component, output row of
                            // component c0)
  const void* X;            // [nfeat][ld]
  const void* y;            // [ld]
  const void* w;            // [ld] or nullptr
  double* slab;             // [nchunks][nrb][GRAD_KT + 2]: loss sum, gradient sums, check statistic
  int64_t ld;
  int64_t nvalid;
  int32_t nchunks;
  int32_t nfeat;
  int32_t rb_rows;          // rows per workgroup (multiple of 64)
  int32_t nrb;
  int32_t chunks_per_group;
  int32_t loss_kind;
  double loss_p0;
  int32_t weighted;
  int32_t max_steps;
  // a derived view's derived-column count (its tangent-zero columns follow at + gd_nd); 0: none
  int32_t gd_nd;
  // row blocks of this launch: blockIdx.x + block0 (slab rows keep their global block index)
  int32_t block0;
  // value-only screening (GMODE_LOSS, KT = 0): a chunk whose block-0 record (written by an earlier
  // launch on the stream) already holds a non-finite check statistic is skipped -- its tree fails
  // did_succeed whatever the other blocks hold
  int32_t screened;
  // per-row modes: out_der[row + j][nvalid] for the components c0 + j < end (the values come from the
  // evaluator, which also decides did_succeed)
  void* out_der;
  // GMODE_LOSS launches of at most GRAD_INLINE chunks pass their (tree, c0) list here, in the kernel
  // arguments (chunks = nullptr): no host-to-device copy on the stream before the launch
  int32_t inl[2 * 96];
};
constexpr int GRAD_INLINE = 96;  // (448 measured the same on C4)
// a chunk is a (tree, c0) pair: the inline list holds GRAD_INLINE of them
static_assert(2 * GRAD_INLINE == sizeof(GradArgs::inl) / sizeof(int32_t), "inline chunk list size");
static_assert(sizeof(GradArgs) <= 4096, "kernel arguments are limited to 4 KB");

// kt = tangent components per chunk: 4 or GRAD_KT (the slab / reduced layout stride is kt + 2)
hipError_t launch_grad(int dtype, int K, int kt, const GradArgs& a, dim3 grid, hipStream_t s);
// per-row modes (GMODE_ROWC / GMODE_ROWF), GRAD_ROW_KT tangents per chunk
hipError_t launch_grad_rows(int dtype, int K, int gmode, const GradArgs& a, dim3 grid, hipStream_t s);
hipError_t launch_grad_reduce(int dtype, int kt, const double* slab, int nrb, int nchunks, double* out, hipStream_t s);
// derived columns of a derived view: Xd[j] = U(X[f]) over ld rows, keys[j] = U << 16 | f (nd <= 32)
hipError_t launch_grad_derive(int dtype, const void* X, void* Xd, int64_t ld, const uint32_t* keys, int nd,
                              hipStream_t s);

}  // namespace srhip
