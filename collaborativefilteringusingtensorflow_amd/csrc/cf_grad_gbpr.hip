// cf_grad_gbpr.hip -- the GBPR gradient kernels' instantiations (launch_grad_m<GBPR>);
// one translation unit per model so that the build compiles them in parallel.
#include "cf_kernels_impl.h"

namespace cfk {

hipError_t launch_grad_gbpr(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    return launch_grad_m<GBPR>(a, nx, s);
}

}  // namespace cfk
