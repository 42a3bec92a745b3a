// Prefill GEMM instantiations for the (QT_Q4_K, QT_Q4_K) weight-format pair (gemm_pf.h); one translation unit
// per pair so the tile set compiles in parallel.
#include "gemm_pf.h"

namespace aios {
template bool pf_launch_fmt<QT_Q4_K, QT_Q4_K>(const GemmQArgs&, int, int, int, hipStream_t);

// timing-anatomy probes of the 256 x 256 Q4_K STORE body (gemm_pf.h PROBE bits); tools only
bool gemm_pf_probe(const GemmQArgs& a, int probe, hipStream_t st) {
  constexpr int NS = pf_slots<QT_Q4_K, QT_Q4_K, 256, 8>();
  constexpr int lds = NS * pf_slot_bytes<QT_Q4_K, QT_Q4_K, 256, 8>();
  if (a.N % 256 || a.K % 256 || a.nseg != 1 || a.seg[0].qtype != QT_Q4_K) return false;
  const dim3 grid((a.N / 256) * ((a.M + 255) / 256)), block(512);
#define PROBE_GO(P, MF) \
  case P + 100 * (MF == 16): \
    hipLaunchKernelGGL((gemm_pf_kernel<QT_Q4_K, QT_Q4_K, 256, 8, NS, GEPI_STORE, P, MF>), grid, block, lds, st, a); \
    return true;
  // probe + 100: the 16x16x32 body; probe + 200: the 4-wave pf4 body (256 x 256); + 300: pf8
  if (probe >= 300) {
    constexpr int lds8 = pf8_lds_bytes<QT_Q4_K, QT_Q4_K, 256>();
    const dim3 g8((a.N / 256) * ((a.M + 255) / 256)), b8(512);
    switch (probe - 300) {
#define P8_GO(P) case P: hipLaunchKernelGGL((gemm_pf8_kernel<QT_Q4_K, QT_Q4_K, 256, GEPI_STORE, P>), g8, b8, lds8, st, a); return true;
      P8_GO(0) P8_GO(1) P8_GO(4) P8_GO(8) P8_GO(13) P8_GO(64) P8_GO(68) P8_GO(77)
#undef P8_GO
      default: return false;
    }
  }
  if (probe >= 200) {
    constexpr int lds4 = pf4_lds_bytes<QT_Q4_K, QT_Q4_K, 256, 64>();
    const dim3 g4((a.N / 256) * ((a.M + 255) / 256)), b4(256);
    switch (probe - 200) {
#define P4_GO(P) case P: hipLaunchKernelGGL((gemm_pf4_kernel<QT_Q4_K, QT_Q4_K, 256, 64, GEPI_STORE, P>), g4, b4, lds4, st, a); return true;
      P4_GO(0) P4_GO(1) P4_GO(4) P4_GO(8) P4_GO(12) P4_GO(13) P4_GO(16) P4_GO(32) P4_GO(17) P4_GO(33)
#undef P4_GO
      default: return false;
    }
  }
  switch (probe) {
    PROBE_GO(0, 32) PROBE_GO(1, 32) PROBE_GO(4, 32) PROBE_GO(8, 32) PROBE_GO(12, 32) PROBE_GO(13, 32)
    PROBE_GO(0, 16) PROBE_GO(1, 16) PROBE_GO(4, 16) PROBE_GO(13, 16)
    default: return false;
  }
#undef PROBE_GO
}
}  // namespace aios
