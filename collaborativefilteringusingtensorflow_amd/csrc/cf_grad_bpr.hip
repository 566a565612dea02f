// cf_grad_bpr.hip -- the BPR gradient kernels' instantiations (launch_grad_m<BPR>);
// one translation unit per model so that the build compiles them in parallel.
#include "cf_kernels_impl.h"

namespace cfk {

hipError_t launch_grad_bpr(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    return launch_grad_m<BPR>(a, nx, s);
}

}  // namespace cfk
