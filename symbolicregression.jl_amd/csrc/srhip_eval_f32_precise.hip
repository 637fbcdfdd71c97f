// srhip_eval_f32_precise.hip — Float32 precise-mode variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f32_precise(const EvalArgs& a, dim3 g, size_t lds, hipStream_t s) {
  return launch_eval_mode<float, R_F32, MODE_PRECISE>(a, 0, false, g, lds, s);
}
}  // namespace srhip
