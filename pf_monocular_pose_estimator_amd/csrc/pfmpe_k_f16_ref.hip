// pfmpe_k_f16_ref.hip — kernel instantiations for fp16-delta state (fp32 compute), kRngReference.
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(float, kRngReference, __half, )
}  // namespace pfmpe_impl
