// Prefill GEMM instantiations for the Q5_K_M stacks (gemm_pf.h; Q5_K, and Q|K Q5_K + V Q6_K QKV): 128-column
// pf4 tiles reading the GEMV engines' Q5_K planes in place.  One translation unit per format set.
#include "gemm_pf.h"

namespace aios {
template bool pf_launch_fmt<QT_Q5_K, QT_Q5_K>(const GemmQArgs&, int, int, int, hipStream_t);
template bool pf_launch_fmt<QT_Q5_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
}  // namespace aios
