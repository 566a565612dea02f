// cf_grad_amf.hip -- the AMF gradient kernels' instantiations (launch_grad_m<AMF>);
// one translation unit per model so that the build compiles them in parallel.
#include "cf_kernels_impl.h"

namespace cfk {

hipError_t launch_grad_amf(const StepArgs& a, const StepArgs* nx, hipStream_t s) {
    return launch_grad_m<AMF>(a, nx, s);
}

}  // namespace cfk
