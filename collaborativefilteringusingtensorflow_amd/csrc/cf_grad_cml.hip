// cf_grad_cml.hip -- the CML gradient kernels' instantiations (launch_grad_m<CML>);
// one translation unit per model so that the build compiles them in parallel.
#include "cf_kernels_impl.h"

namespace cfk {

hipError_t launch_grad_cml(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    return launch_grad_m<CML>(a, nx, s);
}

}  // namespace cfk
