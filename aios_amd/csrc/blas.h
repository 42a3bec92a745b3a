// Plain library GEMMs for long prefill chunks: bf16 activations x the engine's resident bf16 copy of
// a projection's weights through hipBLASLt, fp32 out (optionally accumulated into the residual).
//
// Why a library GEMM here and nowhere else (round 4, profiles/prefill_blas_r4.txt): at 512-2048-token
// chunks the dequant-fused MFMA GEMM (gemm.hip) spends its VALU re-decoding every Q4_K/Q6_K weight
// tile once per 256-token row block and reached 0.62-0.77 PFLOP/s, while hipBLASLt's bf16 TN GEMM
// on the same shapes runs 1.1-1.4 PFLOP/s (profiles/gemm_vs_torch_r2.jsonl).  With 288 GB of HBM
// per GPU a bf16 copy of the projection weights (14 GB for Mistral-7B) is affordable, so the long
// prefill reads it directly; decode and short prompts keep streaming the quantised bytes (one
// residency of the Q4_K_M weights serves them).  The bf16 values are exactly the dequantised Q4_K /
// Q6_K weights the fused GEMM builds in LDS, so both paths multiply the same operands.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <tuple>

#include "common.h"

namespace aios {

class BlasGemm {
 public:
  explicit BlasGemm(size_t workspace_bytes = 64u << 20);
  ~BlasGemm();
  BlasGemm(const BlasGemm&) = delete;
  BlasGemm& operator=(const BlasGemm&) = delete;
  bool ok() const { return handle_ != nullptr; }
  // C[M][N] (fp32, row stride ldc) = A[M][K] (bf16, row stride lda) . W[N][K]^T (bf16, rows of K)
  // (+ C when accumulate).  Returns false (nothing launched) when hipBLASLt has no algorithm for
  // the shape; the caller then takes its own GEMM.
  bool gemm(const bf16_t* A, int lda, const bf16_t* W, float* C, int ldc, int M, int N, int K, bool accumulate,
            hipStream_t st);

 private:
  struct Plan;
  Plan* plan(int M, int N, int K, int lda, int ldc);
  void* handle_ = nullptr;
  void* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  std::map<std::tuple<int, int, int, int, int>, Plan*> plans_;
};

}  // namespace aios
