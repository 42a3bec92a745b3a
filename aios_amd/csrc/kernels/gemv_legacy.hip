// GEMV instantiations: 32-block formats (Q4_0, Q8_0) and 16-bit float weights (F16, BF16).
#include "gemv_impl.h"
namespace aios {
void gemv_q4_0(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q4_0, QT_Q4_0>(a, st); }
void gemv_q8_0(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_Q8_0, QT_Q8_0>(a, st); }
void gemv_f16(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_F16, QT_F16>(a, st); }
void gemv_bf16(const GemvArgs& a, hipStream_t st) { launch_gemv_pair<QT_BF16, QT_BF16>(a, st); }
bool gemv_bf16_engine_fits(const GemvArgs& a) { return launch_gemv_lds16(a, nullptr, true); }
bool gemv_q4_0_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q4_0, QT_Q4_0>(a, nullptr, true); }
bool gemv_q8_0_engine_fits(const GemvArgs& a) { return launch_gemv_lds<QT_Q8_0, QT_Q8_0>(a, nullptr, true); }
bool gemv_tpf_q4_0(const GemvArgs& a, hipStream_t st) { return launch_gemv_tpf<QT_Q4_0>(a, st); }
bool gemv_tpf_q8_0(const GemvArgs& a, hipStream_t st) { return launch_gemv_tpf<QT_Q8_0>(a, st); }
}  // namespace aios
