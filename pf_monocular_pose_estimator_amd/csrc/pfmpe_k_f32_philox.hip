// pfmpe_k_f32_philox.hip — kernel instantiations for float state, kRngPhilox (one TU per pair: parallel build).
#ifndef PFMPE_RESAMPLE_MIN_WAVES
#define PFMPE_RESAMPLE_MIN_WAVES 6  // k_resample / k_resample_multi: 6 waves per SIMD (pf_kernels.hpp)
#endif
#ifndef PFMPE_RESAMPLE_KEPT_MIN_WAVES
#define PFMPE_RESAMPLE_KEPT_MIN_WAVES 6  // the kept-set k_resample variants (pf_kernels.hpp)
#endif
#ifndef PFMPE_WEIGH_STREAM_MIN_WAVES
#define PFMPE_WEIGH_STREAM_MIN_WAVES 6  // k_weigh_stream: 6 waves per SIMD (85 -> 80 VGPRs)
#endif
#ifndef PFMPE_WEIGH_MIN_WAVES
#define PFMPE_WEIGH_MIN_WAVES 6  // k_propagate_weigh: >= 6 waves per SIMD (12/16-marker instances)
#endif
#ifndef PFMPE_WEIGH_PK_MIN_WAVES
#define PFMPE_WEIGH_PK_MIN_WAVES 4  // k_weigh_pk<float>: 4 waves per SIMD (135 -> 128 VGPRs, no scratch)
#endif
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngPhilox, float, )
}  // namespace pfmpe_impl
