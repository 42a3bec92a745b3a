// GEMV instantiations: K-quant formats (Q4_K, Q5_K, Q6_K and the Q4_K_M mixed QKV pairs).
#include "gemv_impl.h"
namespace aios {
void gemv_q4k_q4k(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q4_K, QT_Q4_K>(a, st); }
void gemv_q4k_q6k(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q4_K, QT_Q6_K>(a, st); }
bool gemv_q4k_q4k_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q4_K, QT_Q4_K>(a, nullptr, true); }
bool gemv_q4k_q6k_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q4_K, QT_Q6_K>(a, nullptr, true); }
bool gemv_tpf_q4k(const GemvArgs& a, hipStream_t st) { return launch_gemv_tpf<QT_Q4_K>(a, st); }
}  // namespace aios
