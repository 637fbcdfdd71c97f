// srhip_eval_f64_loss.hip — Float64 loss variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f64_loss(const EvalArgs& a, int K, bool xlds, dim3 g, size_t lds, hipStream_t s) {
  return launch_eval_mode<double, R_F64, MODE_LOSS>(a, K, xlds, g, lds, s);
}
}  // namespace srhip
