// pfmpe_k_f32_ref.hip — kernel instantiations for float state, kRngReference (one TU per pair: parallel build).
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngReference, float, )
}  // namespace pfmpe_impl
