// srhip_eval.hip — gfx950 kernels of the batched expression evaluator: the per-tree partial
// reduction, the batching gather, feature statistics, and the launch dispatch of the interpreter
// (eval_kernel, srhip_eval_impl.h), whose variants are instantiated by the translation units
// srhip_eval_{f32,f64}_{loss,pred,precise}.hip, srhip_eval_f32w.hip and srhip_eval_i32.hip.
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {

// Per-tree reduction of the partials, fixed order (deterministic): one wavefront per order slot
// (slab layout of eval_kernel: loss [row block][slot][chunk of the block], check [row block][slot]);
// the loss chunks are summed in chunk order c = 0.. nch-1 (lane-strided, then a fixed shuffle tree),
// whatever the launch's row-block size; results land at the slot's tree index order[slot].
template <typename LT, typename CT, bool CHK_MAX>
__device__ __forceinline__ void reduce_finish(int slot, LT s, CT m, long long rows, const int32_t* __restrict__ order,
                                              LT* __restrict__ out_loss, CT* __restrict__ out_chk,
                                              int64_t* __restrict__ out_rows, const UndecidedList& ul, int chk_inf) {
  const int tree = order[slot];
  if constexpr (CHK_MAX && sizeof(CT) == 4) {
    if (ul.sbound) m = skip_bound_apply(m, ul.sbound + 4 * (int64_t)tree, ul.fbound);
  }
  if (out_loss) out_loss[tree] = s;
  // chk_inf (row shards): a non-finite statistic is stored as +Inf, which RCCL's MAX / SUM across the
  // shards keep (a max that drops NaN operands would lose a failed shard)
  if (out_chk) out_chk[tree] = chk_inf && !__builtin_isfinite((double)m) ? CT(INFINITY) : m;
  if (out_rows) out_rows[tree] = rows;
  if (ul.ulist && out_chk) {
    bool und;
    if constexpr (CHK_MAX) {
      // exact comparison of chk x rows with 2^127 - 2^102 (the host's long double test)
      const double c = (double)m, p = c * ul.rows, e = __builtin_fma(c, ul.rows, -p), h = 0x1.ffffffp126;
      und = __builtin_isfinite(c) && (p > h || (p == h && e >= 0.0));
    } else {
      und = __builtin_isfinite((double)m) && (double)m >= 0x1p511;
    }
    if (und) {
      const int u = atomicAdd(ul.ulist, 1);
      if (u < ul.umax) ul.ulist[1 + u] = tree;
    }
  }
}

template <typename LT, typename CT, bool CHK_MAX>
__global__ __launch_bounds__(256) void reduce_kernel(const LT* __restrict__ slab_loss, int nch, int cpb,
                                                     const CT* __restrict__ slab_chk, int nrb, int nslots,
                                                     const int32_t* __restrict__ order, LT* __restrict__ out_loss,
                                                     CT* __restrict__ out_chk, const int32_t* __restrict__ slab_rows,
                                                     int64_t* __restrict__ out_rows, UndecidedList ul, int chk_inf,
                                                     int32_t* __restrict__ items_done, int64_t* __restrict__ out_items) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  // a persistent launch's evaluated-item count (its workgroups' sum): reported, then cleared for the
  // context's next persistent launch (this kernel runs after the interpreter on the stream)
  if (items_done && blockIdx.x == 0 && threadIdx.x == 0) {
    *out_items = *items_done;
    *items_done = 0;
  }
  if (slot >= nslots) return;
  LT s = 0;
  CT m = 0;
  long long rows = 0;
  // The same sequential per-lane order as a plain strided loop (lane l adds chunks l, l + 64, ...:
  // the bits every launch form reproduces), with RB_BATCH independent loads issued before their adds:
  // a strided loop waited out one memory latency per iteration (16 per lane for C2's 977 chunks).
  constexpr int RB_BATCH = 16;
  if (slab_loss)
    for (int c0 = lane; c0 < nch; c0 += 64 * RB_BATCH) {
      LT v[RB_BATCH];
      UNR for (int j = 0; j < RB_BATCH; ++j) {
        const int c = c0 + 64 * j;
        v[j] = c < nch ? slab_loss[((int64_t)(c / cpb) * nslots + slot) * cpb + c % cpb] : LT(0);
      }
      UNR for (int j = 0; j < RB_BATCH; ++j)
        if (c0 + 64 * j < nch) s += v[j];
    }
  for (int i0 = lane; i0 < nrb; i0 += 64 * RB_BATCH) {
    CT cv[RB_BATCH];
    int32_t rv[RB_BATCH];
    UNR for (int j = 0; j < RB_BATCH; ++j) {
      const int i = i0 + 64 * j;
      cv[j] = slab_chk && i < nrb ? slab_chk[(int64_t)i * nslots + slot] : CT(0);
      rv[j] = slab_rows && i < nrb ? slab_rows[(int64_t)i * nslots + slot] : 0;
    }
    UNR for (int j = 0; j < RB_BATCH; ++j) {
      if (i0 + 64 * j >= nrb) break;
      if (slab_chk) {
        if constexpr (CHK_MAX) m = __builtin_elementwise_maximum(m, cv[j]); else m += cv[j];
      }
      if (slab_rows) rows += rv[j];
    }
  }
  UNR for (int o = 32; o > 0; o >>= 1) {
    if (slab_loss) s += __shfl_xor(s, o);
    if constexpr (CHK_MAX) m = __builtin_elementwise_maximum(m, __shfl_xor(m, o));
    else m += __shfl_xor(m, o);
    if (slab_rows) rows += __shfl_xor(rows, o);
  }
  if (lane == 0) reduce_finish<LT, CT, CHK_MAX>(slot, s, m, rows, order, out_loss, out_chk, out_rows, ul, chk_inf);
}

// Row ranges of many loss chunks (a few trees over 10M rows: 9766 chunks, 153 per lane): one wave per
// tree waited out ~20 memory latencies (68 us for two trees).  One workgroup per order slot stages the
// slot's chunk partials into LDS, piece by piece, with all its waves' loads in flight, and wave 0 adds
// them from LDS in reduce_kernel's order (lane l: chunks l, l + 64, ... ascending; then the same
// shuffle tree) -- the same bits; the check statistic (a max) and the row count (an integer sum) do
// not depend on the order and take every thread.
constexpr int RW_PIECE = 4096, RW_THREADS = 1024;
template <typename LT, typename CT, bool CHK_MAX>
__global__ __launch_bounds__(RW_THREADS) void reduce_wide_kernel(const LT* __restrict__ slab_loss, int nch, int cpb,
                                                          const CT* __restrict__ slab_chk, int nrb, int nslots,
                                                          const int32_t* __restrict__ order, LT* __restrict__ out_loss,
                                                          CT* __restrict__ out_chk, const int32_t* __restrict__ slab_rows,
                                                          int64_t* __restrict__ out_rows, UndecidedList ul, int chk_inf,
                                                          int32_t* __restrict__ items_done, int64_t* __restrict__ out_items) {
  __shared__ LT buf[RW_PIECE];
  __shared__ CT wm[RW_THREADS / 64];
  __shared__ long long wr[RW_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = blockIdx.x;
  if (items_done && blockIdx.x == 0 && threadIdx.x == 0) {
    *out_items = *items_done;
    *items_done = 0;
  }
  LT s = 0;
  if (slab_loss)
    for (int base = 0; base < nch; base += RW_PIECE) {
      const int n = min(RW_PIECE, nch - base);
      // (every load of the piece issued before the first store: RW_PIECE / RW_THREADS per thread)
      LT v[RW_PIECE / RW_THREADS];
      UNR for (int j = 0; j < RW_PIECE / RW_THREADS; ++j) {
        const int i = (int)threadIdx.x + RW_THREADS * j, c = base + i;
        v[j] = i < n ? slab_loss[((int64_t)(c / cpb) * nslots + slot) * cpb + c % cpb] : LT(0);
      }
      UNR for (int j = 0; j < RW_PIECE / RW_THREADS; ++j) buf[threadIdx.x + RW_THREADS * j] = v[j];
      __syncthreads();
      if (wave == 0) {
#pragma unroll 16
        for (int i = lane; i < n; i += 64) s += buf[i];
      }
      __syncthreads();
    }
  CT m = 0;
  long long rows = 0;
  for (int i0 = threadIdx.x; i0 < nrb; i0 += RW_THREADS * 16) {
    CT cv[16];
    int32_t rv[16];
    UNR for (int j = 0; j < 16; ++j) {
      const int i = i0 + RW_THREADS * j;
      cv[j] = CHK_MAX && slab_chk && i < nrb ? slab_chk[(int64_t)i * nslots + slot] : CT(0);
      rv[j] = slab_rows && i < nrb ? slab_rows[(int64_t)i * nslots + slot] : 0;
    }
    UNR for (int j = 0; j < 16; ++j) {
      if constexpr (CHK_MAX) m = __builtin_elementwise_maximum(m, cv[j]);
      rows += rv[j];
    }
  }
  if constexpr (!CHK_MAX) {
    // a sum (Float64: sum |v| 2^-512): reduce_kernel's order, staged like the loss
    CT* cb = reinterpret_cast<CT*>(buf);
    constexpr int CP = RW_PIECE * (int)sizeof(LT) / (int)sizeof(CT);
    if (slab_chk)
      for (int base = 0; base < nrb; base += CP) {
        const int n = min(CP, nrb - base);
        CT v[CP / RW_THREADS];
        UNR for (int j = 0; j < CP / RW_THREADS; ++j) {
          const int i = (int)threadIdx.x + RW_THREADS * j;
          v[j] = i < n ? slab_chk[(int64_t)(base + i) * nslots + slot] : CT(0);
        }
        UNR for (int j = 0; j < CP / RW_THREADS; ++j) cb[threadIdx.x + RW_THREADS * j] = v[j];
        __syncthreads();
        if (wave == 0) {
#pragma unroll 16
          for (int i = lane; i < n; i += 64) m += cb[i];
        }
        __syncthreads();
      }
  }
  UNR for (int o = 32; o > 0; o >>= 1) {
    if constexpr (CHK_MAX) m = __builtin_elementwise_maximum(m, __shfl_xor(m, o));
    rows += __shfl_xor(rows, o);
  }
  if (lane == 0) {
    wm[wave] = m;
    wr[wave] = rows;
  }
  __syncthreads();
  if (wave != 0) return;
  UNR for (int o = 32; o > 0; o >>= 1) {
    if (slab_loss) s += __shfl_xor(s, o);
    if constexpr (!CHK_MAX) m += __shfl_xor(m, o);
  }
  if (lane == 0) {
    rows = wr[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      if constexpr (CHK_MAX) m = __builtin_elementwise_maximum(m, wm[w]);
      rows += wr[w];
    }
    reduce_finish<LT, CT, CHK_MAX>(slot, s, m, rows, order, out_loss, out_chk, out_rows, ul, chk_inf);
  }
}

// The listed trees' per-operator precise sums over the row blocks, one wave per (tree, operator)
// item: lane l adds row blocks l, l + 64, ... with a compensated (TwoSum) accumulator -- every load
// of the item in flight at once -- and the 64 (sum, compensation) pairs are combined by a fixed xor
// butterfly of double-double additions; results to coherent host memory.  The grid is sized for the
// precise launch's groups; its waves stride over the items of the count read on the device (up to the
// list's capacity umax); the last workgroup to finish resets the list for the next launch on the
// stream (ulist[1 + PRECISE_DONE_SLOT] counts finished workgroups).
__device__ __forceinline__ void two_sum_acc(double& s, double& c, double x) {
  const double t = s + x, bp = t - s;
  c += (s - (t - bp)) + (x - bp);
  s = t;
}
__global__ __launch_bounds__(256) void precise_reduce_kernel(const double* __restrict__ slab, int nrb, int stride,
                                                             int32_t* __restrict__ ulist, int umax, int done_slot,
                                                             int32_t* __restrict__ out_list, double* __restrict__ out) {
  const int cnt = __hip_atomic_load(ulist, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nu = min(cnt, umax);
  const int lane = threadIdx.x & 63;
  for (int item = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); item < nu * stride;
       item += gridDim.x * (blockDim.x / 64)) {
    const double* src = slab + (int64_t)item * nrb;
    double s = 0.0, c = 0.0;
    constexpr int PB = 8;
    for (int b0 = lane; b0 < nrb; b0 += 64 * PB) {
      double xv[PB];
      UNR for (int j = 0; j < PB; ++j) xv[j] = b0 + 64 * j < nrb ? src[b0 + 64 * j] : 0.0;
      UNR for (int j = 0; j < PB; ++j)
        if (b0 + 64 * j < nrb) two_sum_acc(s, c, xv[j]);
    }
    UNR for (int o = 1; o < 64; o <<= 1) {
      const double s2 = __shfl_xor(s, o), c2 = __shfl_xor(c, o);
      // (s, c) + (s2, c2) in an order that does not depend on which lane computes it
      const double a = lane & o ? s2 : s, b = lane & o ? s : s2;
      const double t = a + b, bp = t - a, e = (a - (t - bp)) + (b - bp);
      c = (lane & o ? c2 + c : c + c2) + e;
      s = t;
    }
    if (lane == 0) out[item] = s + c;
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < nu; i += blockDim.x) out_list[1 + i] = ulist[1 + i];
  if (blockIdx.x == 0 && threadIdx.x == 0) out_list[0] = cnt;
  __syncthreads();
  // (every wave's read of the count completed before its value was used, so no fence: the last
  // workgroup's reset cannot overtake another workgroup's read)
  if (threadIdx.x == 0) {
    if (atomicAdd(ulist + 1 + done_slot, 1) == (int)gridDim.x - 1) {
      __hip_atomic_store(ulist + 1 + done_slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ulist, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// View of a dataset through row indices (batching: src/LossFunctions.jl:36-42,114-127):
// dst[f][i] = src[f][idx[i]] for i < m; rows m..ld_dst-1 replicate row idx[m-1]; w pad = 0.
template <typename T>
__global__ void gather_kernel(const T* __restrict__ X, const T* __restrict__ y, const T* __restrict__ w, int64_t ld_src,
                              int nfeat, const int64_t* __restrict__ idx, int64_t m, int64_t ld_dst, T* __restrict__ Xd,
                              T* __restrict__ yd, T* __restrict__ wd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ld_dst) return;
  const bool pad = i >= m;
  const int64_t j = idx[pad ? m - 1 : i];
  for (int f = 0; f < nfeat; ++f) Xd[(int64_t)f * ld_dst + i] = X[(int64_t)f * ld_src + j];
  if (y) yd[i] = y[j];
  if (w) wd[i] = pad ? T(0) : w[j];
}

// Per-feature statistics over the first m rows, for DynamicExpressions' feature-array checks
// (isfinite(sum(X[f, :]))): count of non-finite entries and the f64 sum (Float64 data: sum of
// x * 2^-64 so that it cannot overflow).  grid = (nb row chunks, nfeat): block (b, f) folds chunk b
// of column f into part[f * nb + b]; feature_stats_final folds the nb partials of a feature in
// chunk order (a fixed order: the result does not depend on scheduling).
template <typename T>
__global__ __launch_bounds__(256) void feature_stats_kernel(const T* __restrict__ X, int64_t ld, int64_t m,
                                                            int64_t chunk, FeatStat* __restrict__ part) {
  const int f = blockIdx.y, b = blockIdx.x, nb = gridDim.x;
  const T* col = X + (int64_t)f * ld;
  const int64_t lo = (int64_t)b * chunk, hi = min(m, lo + chunk);
  double s = 0.0, mx = 0.0;
  unsigned long long bad = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const T v = col[i];
    if (!m_isfinite(v)) {
      bad++;
    } else {
      s += sizeof(T) == 8 ? (double)v * 0x1p-64 : (double)v;
      mx = fmax(mx, fabs((double)v));
    }
  }
  __shared__ double ss[256], sm[256];
  __shared__ unsigned long long sb[256];
  ss[threadIdx.x] = s;
  sm[threadIdx.x] = mx;
  sb[threadIdx.x] = bad;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      ss[threadIdx.x] += ss[threadIdx.x + o];
      sm[threadIdx.x] = fmax(sm[threadIdx.x], sm[threadIdx.x + o]);
      sb[threadIdx.x] += sb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[(int64_t)f * nb + b].sum = ss[0];
    part[(int64_t)f * nb + b].nonfinite = (long long)sb[0];
    part[(int64_t)f * nb + b].maxabs = sm[0];
  }
}
__global__ void feature_stats_final(const FeatStat* __restrict__ part, int nb, int nfeat, FeatStat* __restrict__ out) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfeat) return;
  double s = 0.0, mx = 0.0;
  long long bad = 0;
  for (int b = 0; b < nb; ++b) {
    s += part[(int64_t)f * nb + b].sum;
    bad += part[(int64_t)f * nb + b].nonfinite;
    mx = fmax(mx, part[(int64_t)f * nb + b].maxabs);
  }
  out[f].sum = s;
  out[f].nonfinite = bad;
  out[f].maxabs = mx;
}

// ------------------------------------------------------------------------------------------------
// host-side launchers (called from srhip_host.cpp)
// ------------------------------------------------------------------------------------------------
int rows_per_lane(int dtype) { return dtype == SRHIP_F64 ? R_F64 : R_F32; }

int pick_rows_per_lane(int dtype, int K, int mode, int64_t m) {
  // SRHIP_NO_WIDE=1 (tuning runs): never the R = 16 variant
  static const bool no_wide = [] { const char* e = getenv("SRHIP_NO_WIDE"); return e && *e && *e != '0'; }();
  if (!no_wide && dtype == SRHIP_F32 && K <= 2 && mode != MODE_PRECISE && m >= WIDE_MIN_ROWS && R_F32_WIDE != R_F32)
    return R_F32_WIDE;
  return rows_per_lane(dtype);
}

hipError_t launch_eval(int dtype, const EvalArgs& a, int R, int K, int mode, bool xlds, dim3 grid, size_t lds,
                       hipStream_t s) {
  if (R != pick_rows_per_lane(dtype, K, mode, a.nvalid)) return hipErrorInvalidValue;
  if (R == R_F32_WIDE && R != R_F32) {  // Float32, K = 2, loss or prediction
    if (mode != MODE_LOSS && mode != MODE_PRED) return hipErrorInvalidValue;
    return launch_eval_f32w(a, mode, xlds, grid, lds, s);
  }
  switch (dtype) {
    case SRHIP_F32:
      return mode == MODE_LOSS ? launch_eval_f32_loss(a, K, xlds, grid, lds, s)
           : mode == MODE_PRED ? launch_eval_f32_pred(a, K, xlds, grid, lds, s)
                               : launch_eval_f32_precise(a, grid, lds, s);
    case SRHIP_F64:
      return mode == MODE_LOSS ? launch_eval_f64_loss(a, K, xlds, grid, lds, s)
           : mode == MODE_PRED ? launch_eval_f64_pred(a, K, xlds, grid, lds, s)
                               : launch_eval_f64_precise(a, grid, lds, s);
    case SRHIP_I32:
      return mode == MODE_PRECISE ? hipErrorInvalidValue : launch_eval_i32(a, K, mode, xlds, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_precise_reduce(const double* slab, int nrb, int stride, int32_t* ulist, int umax, int groups,
                                 int done_slot, int32_t* out_list, double* out, hipStream_t s) {
  const int items = std::max(1, std::min(umax, groups) * stride);
  hipLaunchKernelGGL(precise_reduce_kernel, dim3((items + 3) / 4), dim3(256), 0, s, slab, nrb, stride, ulist, umax,
                     done_slot, out_list, out);
  return hipGetLastError();
}

hipError_t launch_reduce(int dtype, const void* slab_loss, int nch, int cpb, const void* slab_chk, int nrb, int nslots,
                         const int32_t* order, void* out_loss, void* out_chk, hipStream_t s, const int32_t* slab_rows,
                         int64_t* out_rows, const UndecidedList& ul, bool chk_inf, int32_t* items_done,
                         int64_t* out_items) {
  dim3 grid((nslots + 3) / 4), block(256);
  // more than one batch of loads per lane: a workgroup per slot (reduce_wide_kernel, the same bits)
  const char* nw = getenv("SRHIP_NO_WIDE_REDUCE");  // (read per launch: the tests toggle it)
  if (!(nw && *nw && *nw != '0') && std::max(nch, nrb) > 64 * 16) {
    const dim3 g(nslots), wb(RW_THREADS);
    switch (dtype) {
      case SRHIP_F32:
        hipLaunchKernelGGL((reduce_wide_kernel<double, float, true>), g, wb, 0, s, (const double*)slab_loss, nch, cpb,
                           (const float*)slab_chk, nrb, nslots, order, (double*)out_loss, (float*)out_chk, slab_rows,
                           out_rows, ul, (int)chk_inf, items_done, out_items);
        break;
      case SRHIP_F64:
        hipLaunchKernelGGL((reduce_wide_kernel<double, double, false>), g, wb, 0, s, (const double*)slab_loss, nch,
                           cpb, (const double*)slab_chk, nrb, nslots, order, (double*)out_loss, (double*)out_chk,
                           slab_rows, out_rows, ul, (int)chk_inf, items_done, out_items);
        break;
      case SRHIP_I32:
        hipLaunchKernelGGL((reduce_wide_kernel<long long, float, true>), g, wb, 0, s, (const long long*)slab_loss,
                           nch, cpb, (const float*)nullptr, nrb, nslots, order, (long long*)out_loss, (float*)nullptr,
                           slab_rows, out_rows, UndecidedList(), 0, items_done, out_items);
        break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (dtype) {
    case SRHIP_F32:
      hipLaunchKernelGGL((reduce_kernel<double, float, true>), grid, block, 0, s, (const double*)slab_loss, nch, cpb,
                         (const float*)slab_chk, nrb, nslots, order, (double*)out_loss, (float*)out_chk, slab_rows,
                         out_rows, ul, (int)chk_inf, items_done, out_items);
      break;
    case SRHIP_F64:
      hipLaunchKernelGGL((reduce_kernel<double, double, false>), grid, block, 0, s, (const double*)slab_loss, nch, cpb,
                         (const double*)slab_chk, nrb, nslots, order, (double*)out_loss, (double*)out_chk, slab_rows,
                         out_rows, ul, (int)chk_inf, items_done, out_items);
      break;
    case SRHIP_I32:
      hipLaunchKernelGGL((reduce_kernel<long long, float, true>), grid, block, 0, s, (const long long*)slab_loss, nch,
                         cpb, (const float*)nullptr, nrb, nslots, order, (long long*)out_loss, (float*)nullptr,
                         slab_rows, out_rows, UndecidedList(), 0, items_done, out_items);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gather(int dtype, const void* X, const void* y, const void* w, int64_t ld_src, int nfeat,
                         const int64_t* idx, int64_t m, int64_t ld_dst, void* Xd, void* yd, void* wd, hipStream_t s) {
  dim3 block(256), grid((unsigned)((ld_dst + 255) / 256));
  switch (dtype) {
    case SRHIP_F32:
      hipLaunchKernelGGL(gather_kernel<float>, grid, block, 0, s, (const float*)X, (const float*)y, (const float*)w,
                         ld_src, nfeat, idx, m, ld_dst, (float*)Xd, (float*)yd, (float*)wd);
      break;
    case SRHIP_F64:
      hipLaunchKernelGGL(gather_kernel<double>, grid, block, 0, s, (const double*)X, (const double*)y,
                         (const double*)w, ld_src, nfeat, idx, m, ld_dst, (double*)Xd, (double*)yd, (double*)wd);
      break;
    case SRHIP_I32:
      hipLaunchKernelGGL(gather_kernel<int32_t>, grid, block, 0, s, (const int32_t*)X, (const int32_t*)y,
                         (const int32_t*)w, ld_src, nfeat, idx, m, ld_dst, (int32_t*)Xd, (int32_t*)yd, (int32_t*)wd);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_feature_stats(int dtype, const void* X, int64_t ld, int64_t m, int nfeat, FeatStat* out,
                                hipStream_t s) {
  if (nfeat <= 0) return hipSuccess;
  // out holds nfeat results followed by nfeat * FEAT_STAT_BLOCKS partials (feature_stats_scratch)
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(FEAT_STAT_BLOCKS, m / 65536));
  const int64_t chunk = (m + nb - 1) / nb;
  FeatStat* part = out + nfeat;
  const dim3 grid(nb, nfeat), block(256);
  switch (dtype) {
    case SRHIP_F32:
      hipLaunchKernelGGL(feature_stats_kernel<float>, grid, block, 0, s, (const float*)X, ld, m, chunk, part);
      break;
    case SRHIP_F64:
      hipLaunchKernelGGL(feature_stats_kernel<double>, grid, block, 0, s, (const double*)X, ld, m, chunk, part);
      break;
    default: return hipSuccess;
  }
  hipLaunchKernelGGL(feature_stats_final, dim3((nfeat + 63) / 64), dim3(64), 0, s, (const FeatStat*)part, nb, nfeat, out);
  return hipGetLastError();
}

}  // namespace srhip
