// pfmpe_k_f64_philox.hip — kernel instantiations for double state, kRngPhilox (one TU per pair: parallel build).
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(double, kRngPhilox, double, )
}  // namespace pfmpe_impl
