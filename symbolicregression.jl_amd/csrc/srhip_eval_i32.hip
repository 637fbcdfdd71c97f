// srhip_eval_i32.hip — Int32 variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_i32(const EvalArgs& a, int K, int mode, bool xlds, dim3 g, size_t lds, hipStream_t s) {
  return mode == MODE_LOSS ? launch_eval_mode<int32_t, R_F32, MODE_LOSS>(a, K, xlds, g, lds, s)
                           : launch_eval_mode<int32_t, R_F32, MODE_PRED>(a, K, xlds, g, lds, s);
}
}  // namespace srhip
