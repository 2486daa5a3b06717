// pfmpe_k_f32_philox.hip — kernel instantiations for float state, kRngPhilox (one TU per pair: parallel build).
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngPhilox, float, )
}  // namespace pfmpe_impl
