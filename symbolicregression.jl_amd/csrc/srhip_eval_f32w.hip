// srhip_eval_f32w.hip — wide Float32 (R = 16, K = 2: the C2 / C3 kernel) variant slice of the interpreter (srhip_eval_impl.h).
#include "srhip_eval_impl.h"
#include "srhip_eval_variants.h"

namespace srhip {
hipError_t launch_eval_f32w(const EvalArgs& a, int mode, bool xlds, dim3 g, size_t lds, hipStream_t s) {
  if (mode == MODE_LOSS)
    return xlds ? launch_eval_t<float, R_F32_WIDE, 2, MODE_LOSS, true>(a, g, lds, s)
                : launch_eval_t<float, R_F32_WIDE, 2, MODE_LOSS, false>(a, g, lds, s);
  return xlds ? launch_eval_t<float, R_F32_WIDE, 2, MODE_PRED, true>(a, g, lds, s)
              : launch_eval_t<float, R_F32_WIDE, 2, MODE_PRED, false>(a, g, lds, s);
}
}  // namespace srhip
