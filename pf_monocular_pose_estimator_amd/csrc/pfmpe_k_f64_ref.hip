// pfmpe_k_f64_ref.hip — kernel instantiations for double state, kRngReference (one TU per pair: parallel build).
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(double, kRngReference, double, )
}  // namespace pfmpe_impl
