// srhip_grad.h — argument block and launchers of the constant-gradient kernels (srhip_grad.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srhip_isa.h"

namespace srhip {

constexpr int GRAD_WAVES = 8;  // wavefronts per workgroup
constexpr int GRAD_KT = 8;     // tangent components per pass (constants per chunk)

struct GradArgs {
  const Ins* code;          // gradient programs of all trees
  const int32_t* prog_off;  // [ntrees]
  const int32_t* chunks;    // [nchunks][2]: (tree, first constant)
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
};

// kt = tangent components per chunk: 4 or GRAD_KT (the slab / reduced layout stride is kt + 2)
hipError_t launch_grad(int dtype, int K, int kt, const GradArgs& a, dim3 grid, hipStream_t s);
hipError_t launch_grad_reduce(int dtype, int kt, const double* slab, int nrb, int nchunks, double* out, hipStream_t s);

}  // namespace srhip
