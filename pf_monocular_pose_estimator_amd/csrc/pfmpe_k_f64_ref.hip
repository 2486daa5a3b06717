// pfmpe_k_f64_ref.hip — kernel instantiations for double state, kRngReference (one TU per pair: parallel build).
#define PFMPE_FRAME2_MIN_WAVES 3  // k_frame2: one launch up to 512 blocks (pf_kernels.hpp)
#include "pfmpe_ctx.hpp"

namespace pfmpe_impl {
using namespace pfmpe;
PFMPE_DECLARE_INSTANCE(double, kRngReference, double, )
}  // namespace pfmpe_impl
