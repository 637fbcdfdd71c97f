// srhip_kernels.h — kernel argument blocks and launcher declarations (host <-> srhip_eval.hip and the srhip_eval_<slice>.hip variant units).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srhip_isa.h"

namespace srhip {

#ifndef SRHIP_EVAL_WAVES
#define SRHIP_EVAL_WAVES 8
#endif
constexpr int EVAL_WAVES = SRHIP_EVAL_WAVES;  // wavefronts per workgroup of the interpreter kernel
// ... except the wide Float32 variant (R = 16, K = 2: the C2 / C3 kernel), which runs 16-wave
// workgroups, one per CU, over 4096-row blocks: twice the rows per staged block and per tree (the
// early exit of failed trees saves more of each block), the same 4 waves per SIMD (C2, one MI355X:
// 1.47 -> 1.34 ms)
constexpr int EVAL_WAVES_WIDE = 16;
constexpr int eval_waves(int R, int K) { return (R == 16 && K <= 2) ? EVAL_WAVES_WIDE : EVAL_WAVES; }
constexpr int EVAL_WAVES_MAX = EVAL_WAVES_WIDE > EVAL_WAVES ? EVAL_WAVES_WIDE : EVAL_WAVES;
#ifndef SRHIP_R_F32
#define SRHIP_R_F32 8
#endif
constexpr int R_F32 = SRHIP_R_F32;  // rows per lane per dispatch, 4-byte types
constexpr int R_F64 = 4;       // rows per lane per dispatch, Float64
// Float32 trees whose stack fits K = 2 on datasets of at least WIDE_MIN_ROWS rows run with twice
// the rows per lane: the per-instruction dispatch cost is paid once per 16 rows (121 VGPRs,
// 4 waves per SIMD; the VALU-bound operators are unaffected, the cheap ones get ~20 % faster).
constexpr int R_F32_WIDE = 16;
constexpr int64_t WIDE_MIN_ROWS = 4096;
constexpr int ROW_ALIGN = 4096;  // device datasets are padded to a multiple of this many rows
constexpr int MODE_LOSS = 0, MODE_PRED = 1, MODE_PRECISE = 2;
// Loss partials are kept per fixed chunk of rows (not per workgroup row block): every lane adds
// its rows of a chunk in the same order whatever R, K, row-block size or program (derived columns
// or not) evaluates the tree, so a tree's loss on a dataset is one bit pattern in every launch.
// Row blocks are whole chunks.
constexpr int LOSS_CHUNK_4B = 1024, LOSS_CHUNK_8B = 256;
inline int loss_chunk(int dtype) { return dtype == SRHIP_F64 ? LOSS_CHUNK_8B : LOSS_CHUNK_4B; }

struct FeatStat {
  double sum;           // f64 sum (Float64 data: sum of x * 2^-64)
  long long nonfinite;  // count of Inf/NaN entries
  double maxabs;        // max |x| over the finite entries (round 6: the Float32 interpreter's +/- bound)
};
// launch_feature_stats splits each column into at most FEAT_STAT_BLOCKS row chunks; its output
// buffer holds the nfeat results followed by the partials.
constexpr int FEAT_STAT_BLOCKS = 64;
inline size_t feature_stats_scratch(int64_t nfeat) { return (size_t)(nfeat < 1 ? 1 : nfeat) * (1 + FEAT_STAT_BLOCKS); }

struct EvalArgs {
  const Ins* code;          // all trees' bytecode
  const int32_t* prog_off;  // [ntrees] first instruction of each tree
  const int32_t* order;     // [ntrees] processing order (grouped, cost-sorted)
  const void* X;            // [>= nfeat][ld] SoA, padded (the first nfeat columns are staged)
  const void* y;            // [ld] (nullptr for prediction-only)
  const void* w;            // [ld] or nullptr
  void* slab_loss;          // [nrb][ntrees][rb_rows / loss chunk] loss partials per row chunk, by order slot
                            // (double; int64 for Int32)
  void* slab_chk;           // [nrb][ntrees] check partials by order slot (float max|v| / double sum|v|*2^-512)
  void* out_pred;           // [ntrees][nvalid] (MODE_PRED)
  void* slab_prec;          // [n][prec_stride][nrb] double (MODE_PRECISE)
  int64_t ld;               // padded rows of X / y / w
  int64_t nvalid;           // rows evaluated
  int32_t ntrees;
  int32_t nfeat;
  int32_t rb_rows;          // rows per workgroup (multiple of 64*R)
  int32_t nrb;              // row blocks
  int32_t nch;              // loss chunks: ceil(nvalid / loss_chunk)
  int32_t cpb;              // loss chunks per row block (rb_rows / loss_chunk)
  int32_t trees_per_group;  // trees per grid.y group (group_off == nullptr)
  const int32_t* group_off; // [grid.y + 1] first order slot of each group, or nullptr (uniform groups)
  int32_t loss_kind;
  double loss_p0;
  int32_t weighted;
  int32_t prec_stride;      // operator nodes per tree slot in slab_prec
  int32_t has_y;            // stage y into LDS (MODE_LOSS)
  int32_t max_steps;        // longest tree program (instructions): bounds every interpreter loop
  int32_t debug_stop;       // diagnostic early exits (SRHIP_DEBUG_STOP); 0 in normal runs
  int32_t nd;               // derived columns (LDS columns nfeat .. nfeat+nd-1); 0 unless XLDS
  const uint32_t* dspec;    // [nd] (U << 16) | feature of each derived column
  const uint64_t* dmask;    // [program trees] bit d: the tree reads derived column d
  int32_t* dbg;             // SRHIP_TRACE: host-coherent progress words of block (0,0) wave 0, else nullptr
  int32_t early_exit;       // MODE_LOSS: a wave stops a tree's row block once its check statistic is
                            // non-finite (the tree has failed: DynamicExpressions' early return) and
                            // marks the tree failed for the row blocks that have not started it
  int32_t epoch;            // this launch's mark (> 0; fail_flag[slot] == epoch: failed in this launch)
  int32_t* fail_flag;       // [ntrees] by order slot
  // single-row-block launches (nrb == 1, small datasets): each wave finishes its tree's reduction
  // itself, in reduce_kernel's order, and writes the results to these (coherent pinned host) arrays
  // indexed by tree; no reduce launch
  int32_t fused;
  void* fused_loss;         // [program trees] LAccT (MODE_LOSS) or nullptr
  void* fused_chk;          // [program trees] check statistic type, or nullptr (Int32)
  // persistent launches (one tree group, the whole population): grid.x workgroups claim row blocks
  // block0 .. nrb-1 from *block_ctr (zeroed before the launch)
  int32_t persistent;
  int32_t block0;
  int32_t tail_blocks;      // the last tail_blocks row blocks are claimed as tail_slices population slices each
  int32_t tail_slices;
  int32_t grid_interleave;  // grid launches: workgroup (x, y) takes order slots y, y + grid.y, ... (group_off unused)
  int32_t tile_claims;      // a wave claims one (tree, tile) at a time (R = 16 probe; slab_chk / slab_rows zeroed first)
  int32_t block_stride;     // grid launches: workgroup x takes row blocks x, x + grid.x, ... (< nrb)
  int32_t* block_ctr;
  // probe launches (tile_claims): zero_ctr, if set, is the persistent launch's block counter, zeroed
  // by workgroup (0, 0) -- the persistent launch follows on the same stream; and every workgroup zeroes
  // its own (row block, slot) entries of slab_chk / slab_rows before its waves combine into them
  int32_t* zero_ctr;
  // MODE_PRECISE launches over a device-built list of undecided trees (order = the list): the number
  // of listed trees is read here (*dev_count, capped at trees_per_group); each wave zeroes its
  // (tree, row block) slab entries before accumulating into them
  const int32_t* dev_count;
  int32_t wg_waves;         // waves per workgroup (0: the variant's eval_waves; fewer claim the same trees)
  int32_t prec_assign;      // MODE_PRECISE with one tile per (tree, row block): store the per-operator
                            // sums instead of adding to them (no dependent load per operator)
  int32_t* slab_rows;       // [nrb][ntrees] valid rows each (row block, order slot) evaluated, or nullptr
  int64_t* fused_rows;      // fused launches: [program trees] rows evaluated (coherent pinned host), or nullptr
};

int rows_per_lane(int dtype);
// rows per lane of the kernel variant that evaluates a launch (K stack slots, mode, m rows)
int pick_rows_per_lane(int dtype, int K, int mode, int64_t m);
hipError_t launch_eval(int dtype, const EvalArgs& a, int R, int K, int mode, bool xlds, dim3 grid, size_t lds,
                       hipStream_t s);
// per-tree reduction of eval_kernel's slabs: nslots order slots, cpb loss chunks per row block, results
// at out[order[slot]]
// slab_rows (optional): [nrb][nslots] rows evaluated, summed per tree into out_rows (int64)
// The device's share of the did_succeed decision: a tree whose check statistic is finite
// but whose overflow bound reaches half the threshold (Float32: chk x rows >= 2^127 - 2^102 exactly;
// Float64: chk >= 2^511) is appended to ulist (ulist[0] = count, trees from ulist[1], at most umax;
// the count keeps growing past umax) for the precise pass that follows on the stream.
struct UndecidedList {
  int32_t* ulist = nullptr;  // nullptr: no device list (the host decides after the launch)
  int32_t umax = 0;
  double rows = 0.0;
  // Float32 programs (round 6): + and - fold no check statistic in the interpreter.  Per program tree
  // (cM, cF, c0, 0) bounds every +/- output by cM M + cF fbound + c0 (M: the statistic of the folded
  // values, fbound: the features' max |x|, +Inf if any is non-finite; TreeCompiler::skip_bounds); the
  // reduction raises each tree's statistic to that bound (skip_bound_apply) before it is written or
  // tested.  nullptr: no bound (Float64, Int32)
  const float* sbound = nullptr;
  float fbound = 0.0f;
};
// max(M, cM M + cF F + c0) clamped to FLT_MAX for a finite M (a non-finite M stands): a finite bound
// only ever turns a decided tree into an undecided one -- which the exact precise pass then decides --
// and never a finite statistic into a failure.  The same function on the host (fused single-block
// launches) and in the reduction.
__host__ __device__ inline float skip_bound_apply(float M, const float* sb, float F) {
  if (!(sb[0] > 0.0f || sb[1] > 0.0f || sb[2] > 0.0f) || !(M - M == 0.0f)) return M;
  const double fb = sb[1] > 0.0f ? (double)sb[1] * (double)F : 0.0;
  const double bd = (double)sb[0] * (double)M + (fb + (double)sb[2]);
  const double mb = bd > (double)M ? bd : (double)M;
  return mb < (double)__FLT_MAX__ ? (float)mb : __FLT_MAX__;
}
hipError_t launch_reduce(int dtype, const void* slab_loss, int nch, int cpb, const void* slab_chk, int nrb, int nslots,
                         const int32_t* order, void* out_loss, void* out_chk, hipStream_t s,
                         const int32_t* slab_rows = nullptr, int64_t* out_rows = nullptr,
                         const UndecidedList& ul = UndecidedList(), bool chk_inf = false,
                         int32_t* items_done = nullptr, int64_t* out_items = nullptr);
// The precise pass's per-(listed tree, operator) sums over the row blocks (fixed order, compensated),
// written to out (coherent host memory: out_count, then [umax][stride] doubles); the last workgroup
// resets ulist[0] (ulist[1 + done_slot]: its finished-workgroup counter, zero between launches).
hipError_t launch_precise_reduce(const double* slab, int nrb, int stride, int32_t* ulist, int umax, int groups, int done_slot,
                                 int32_t* out_list, double* out, hipStream_t s);
hipError_t launch_gather(int dtype, const void* X, const void* y, const void* w, int64_t ld_src, int nfeat,
                         const int64_t* idx, int64_t m, int64_t ld_dst, void* Xd, void* yd, void* wd, hipStream_t s);
hipError_t launch_feature_stats(int dtype, const void* X, int64_t ld, int64_t m, int nfeat, FeatStat* out,
                                hipStream_t s);

}  // namespace srhip
