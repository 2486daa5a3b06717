// pfmpe_k_f16_ref.hip — kernel instantiations for fp16-delta state (fp32 compute), kRngReference.
#ifndef PFMPE_RESAMPLE_MIN_WAVES
#define PFMPE_RESAMPLE_MIN_WAVES 7  // k_resample: 7 waves per SIMD (pf_kernels.hpp)
#endif
#ifndef PFMPE_WEIGH_STREAM_MIN_WAVES
#define PFMPE_WEIGH_STREAM_MIN_WAVES 6  // k_weigh_stream: 6 waves per SIMD (85 -> 80 VGPRs)
#endif
#ifndef PFMPE_WEIGH_MIN_WAVES
#define PFMPE_WEIGH_MIN_WAVES 6  // k_propagate_weigh: >= 6 waves per SIMD (12/16-marker instances)
#endif
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngReference, __half, )
}  // namespace pfmpe_impl
