// Prefill GEMM instantiations for the (QT_Q4_K, QT_Q6_K) weight-format pair (gemm_pf.h); one translation unit
// per pair so the tile set compiles in parallel.
#include "gemm_pf.h"

namespace aios {
template bool pf_launch_fmt<QT_Q4_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
}  // namespace aios
