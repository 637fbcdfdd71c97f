// srhip_eval_variants.h — launchers of the interpreter's variant slices, one translation unit each
// (srhip_eval_<slice>.hip), so that the slices compile in parallel.
#pragma once
#include "srhip_kernels.h"

namespace srhip {
hipError_t launch_eval_f32_loss(const EvalArgs& a, int K, bool xlds, dim3 grid, size_t lds, hipStream_t s);
hipError_t launch_eval_f32_pred(const EvalArgs& a, int K, bool xlds, dim3 grid, size_t lds, hipStream_t s);
hipError_t launch_eval_f32_precise(const EvalArgs& a, dim3 grid, size_t lds, hipStream_t s);
// Float32, R = R_F32_WIDE, K = 2: MODE_LOSS or MODE_PRED
hipError_t launch_eval_f32w(const EvalArgs& a, int mode, bool xlds, dim3 grid, size_t lds, hipStream_t s);
hipError_t launch_eval_f64_loss(const EvalArgs& a, int K, bool xlds, dim3 grid, size_t lds, hipStream_t s);
hipError_t launch_eval_f64_pred(const EvalArgs& a, int K, bool xlds, dim3 grid, size_t lds, hipStream_t s);
hipError_t launch_eval_f64_precise(const EvalArgs& a, dim3 grid, size_t lds, hipStream_t s);
// Int32: MODE_LOSS or MODE_PRED
hipError_t launch_eval_i32(const EvalArgs& a, int K, int mode, bool xlds, dim3 grid, size_t lds, hipStream_t s);
}  // namespace srhip
