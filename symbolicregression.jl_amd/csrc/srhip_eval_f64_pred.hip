// srhip_eval_f64_pred.hip — Float64 prediction variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f64_pred(const EvalArgs& a, int K, bool xlds, dim3 g, size_t lds, hipStream_t s) {
  return launch_eval_mode<double, R_F64, MODE_PRED>(a, K, xlds, g, lds, s);
}
}  // namespace srhip
