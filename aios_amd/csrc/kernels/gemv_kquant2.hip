// GEMV instantiations: Q6_K (lm_head / ffn_down in Q4_K_M) and Q5_K (Q5_K_M files).
#include "gemv_impl.h"
namespace aios {
void gemv_q6k_q6k(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q6_K, QT_Q6_K>(a, st); }
void gemv_q5k_q5k(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q5_K, QT_Q5_K>(a, st); }
void gemv_q5k_q6k(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q5_K, QT_Q6_K>(a, st); }
bool gemv_q6k_q6k_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q6_K, QT_Q6_K>(a, nullptr, true); }
bool gemv_q5k_q5k_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q5_K, QT_Q5_K>(a, nullptr, true); }
bool gemv_q5k_q6k_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q5_K, QT_Q6_K>(a, nullptr, true); }
bool gemv_tpf_q6k(const GemvArgs& a, hipStream_t st) { return launch_gemv_tpf<QT_Q6_K>(a, st); }
bool gemv_tpf_q5k(const GemvArgs& a, hipStream_t st) { return launch_gemv_tpf<QT_Q5_K>(a, st); }
}  // namespace aios
