// cf_grad_plr.hip -- the tuple-ranking (PRIGP / CPLR) gradient kernels'
// instantiations, in their own translation unit (see cf_grad_bpr.hip).
#include "cf_kernels_impl.h"

namespace cfk {

hipError_t launch_grad_plr_t(const StepArgs& a, hipStream_t s) { return launch_grad_plr(a, s); }

}  // namespace cfk
