// Prefill GEMM instantiations for the 32-weight-block formats Q4_0 and Q8_0 (gemm_pf.h): 128-column pf4
// tiles reading the GEMV engines' planes in place.  One translation unit per format set.
#include "gemm_pf.h"

namespace aios {
template bool pf_launch_fmt<QT_Q4_0, QT_Q4_0>(const GemmQArgs&, int, int, int, hipStream_t);
template bool pf_launch_fmt<QT_Q8_0, QT_Q8_0>(const GemmQArgs&, int, int, int, hipStream_t);
}  // namespace aios
