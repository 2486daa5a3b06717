// pfmpe_k_f16_philox.hip — kernel instantiations for fp16-delta state (fp32 compute), kRngPhilox.
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngPhilox, __half, )
}  // namespace pfmpe_impl
