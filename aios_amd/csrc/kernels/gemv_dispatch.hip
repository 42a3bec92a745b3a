// Host dispatcher: (segment-0 format, last-segment format) -> kernel instantiation.
#include <stdexcept>
#include <string>

#include "../gemv.h"

namespace aios {
void gemv_q4k_q4k(const GemvArgs&, hipStream_t);
void gemv_q4k_q6k(const GemvArgs&, hipStream_t);
void gemv_q6k_q6k(const GemvArgs&, hipStream_t);
void gemv_q5k_q5k(const GemvArgs&, hipStream_t);
void gemv_q5k_q6k(const GemvArgs&, hipStream_t);
void gemv_q4_0(const GemvArgs&, hipStream_t);
void gemv_q8_0(const GemvArgs&, hipStream_t);
void gemv_f16(const GemvArgs&, hipStream_t);
void gemv_bf16(const GemvArgs&, hipStream_t);

bool gemv_q4k_q4k_engine_fits(const GemvArgs&);
bool gemv_q4k_q6k_engine_fits(const GemvArgs&);
bool gemv_q6k_q6k_engine_fits(const GemvArgs&);
bool gemv_q5k_q5k_engine_fits(const GemvArgs&);
bool gemv_q5k_q6k_engine_fits(const GemvArgs&);
bool gemv_q4_0_engine_fits(const GemvArgs&);
bool gemv_q8_0_engine_fits(const GemvArgs&);

// Whether the B-row LDS-DMA engine serves these args (B = 1..4, int8 activations, the shape's LDS
// plan fits 160 KB).  16-bit weights never take the engine and report true (their B-row kernels are
// the only GEMV path).  The engine's batched-decode path choice asks this per projection.
bool gemv_engine_fits(const GemvArgs& a) {
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  if (qt0 == QT_F16 || qt0 == QT_BF16) return true;
  if (qt0 == qt1) {
    switch (qt0) {
      case QT_Q4_K: return gemv_q4k_q4k_engine_fits(a);
      case QT_Q6_K: return gemv_q6k_q6k_engine_fits(a);
      case QT_Q5_K: return gemv_q5k_q5k_engine_fits(a);
      case QT_Q4_0: return gemv_q4_0_engine_fits(a);
      case QT_Q8_0: return gemv_q8_0_engine_fits(a);
    }
  } else if (qt1 == QT_Q6_K) {
    if (qt0 == QT_Q4_K) return gemv_q4k_q6k_engine_fits(a);
    if (qt0 == QT_Q5_K) return gemv_q5k_q6k_engine_fits(a);
  }
  return false;
}

bool gemv_tpf_q4k(const GemvArgs&, hipStream_t);
bool gemv_tpf_q6k(const GemvArgs&, hipStream_t);
bool gemv_tpf_q5k(const GemvArgs&, hipStream_t);
bool gemv_tpf_q4_0(const GemvArgs&, hipStream_t);
bool gemv_tpf_q8_0(const GemvArgs&, hipStream_t);

// EPI_TP_RESID (the TP all-reduce in the GEMV epilogue): launched by the row-pair kernel, or false
// with nothing launched (format, shape or stage capacity outside it) -- the caller then runs the
// plain GEMV and a separate all-reduce
bool launch_gemv_tp_fused(const GemvArgs& a, hipStream_t st) {
  if (a.nseg != 1 || a.epi != EPI_TP_RESID) return false;
  switch (a.seg[0].qtype) {
    case QT_Q4_K: return gemv_tpf_q4k(a, st);
    case QT_Q6_K: return gemv_tpf_q6k(a, st);
    case QT_Q5_K: return gemv_tpf_q5k(a, st);
    case QT_Q4_0: return gemv_tpf_q4_0(a, st);
    case QT_Q8_0: return gemv_tpf_q8_0(a, st);
  }
  return false;
}

bool gemv_supports(int qt0, int qt1) {
  if (qt0 == qt1)
    return qt0 == QT_Q4_K || qt0 == QT_Q6_K || qt0 == QT_Q5_K || qt0 == QT_Q4_0 || qt0 == QT_Q8_0 ||
           qt0 == QT_F16 || qt0 == QT_BF16;
  return (qt0 == QT_Q4_K || qt0 == QT_Q5_K) && qt1 == QT_Q6_K;
}

void launch_gemv(const GemvArgs& a, hipStream_t st) {
  if (a.nseg < 1 || a.nseg > GEMV_MAX_SEGS) throw std::runtime_error("gemv: bad segment count");
  if (a.B < 1 || a.B > 8) throw std::runtime_error("gemv: batch must be 1..8");
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  for (int s = 0; s + 1 < a.nseg; ++s)
    if (a.seg[s].qtype != qt0) throw std::runtime_error("gemv: only the last segment may differ in format");
  for (int s = 0; s < a.nseg; ++s) {
    if (a.seg[s].cols != a.K) throw std::runtime_error("gemv: segment K mismatch");
    if (a.seg_row0[s] % 8) throw std::runtime_error("gemv: segment boundary must be a multiple of 8 rows");
  }
  if (a.N % 2) throw std::runtime_error("gemv: N must be even");
  if (a.K % 16) throw std::runtime_error("gemv: K must be a multiple of 16");
  if (qt0 == qt1) {
    switch (qt0) {
      case QT_Q4_K: return gemv_q4k_q4k(a, st);
      case QT_Q6_K: return gemv_q6k_q6k(a, st);
      case QT_Q5_K: return gemv_q5k_q5k(a, st);
      case QT_Q4_0: return gemv_q4_0(a, st);
      case QT_Q8_0: return gemv_q8_0(a, st);
      case QT_F16: return gemv_f16(a, st);
      case QT_BF16: return gemv_bf16(a, st);
    }
  } else if (qt1 == QT_Q6_K) {
    if (qt0 == QT_Q4_K) return gemv_q4k_q6k(a, st);
    if (qt0 == QT_Q5_K) return gemv_q5k_q6k(a, st);
  }
  throw std::runtime_error("gemv: unsupported format pair " + std::to_string(qt0) + "/" + std::to_string(qt1));
}
}  // namespace aios
