// srhip_eval_f64_precise.hip — Float64 precise-mode variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f64_precise(const EvalArgs& a, dim3 g, size_t lds, hipStream_t s) {
  return launch_eval_mode<double, R_F64, MODE_PRECISE>(a, 0, false, g, lds, s);
}
}  // namespace srhip
