// srhip_eval_f32x.hip — extra-wide Float32 (R = 32, K = 2: the persistent C2 / C3 loss launch, SRHIP_XWIDE)
// variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f32x(const EvalArgs& a, dim3 g, size_t lds, hipStream_t s) {
  return launch_eval_t<float, R_F32_XWIDE, 2, MODE_LOSS, true>(a, g, lds, s);
}
}  // namespace srhip
