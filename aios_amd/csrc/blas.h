// Plain bf16 library GEMM (hipBLASLt) for the prefill / large-batch projections on weights
// dequantised once at load into resident bf16 copies (288 GB of HBM holds both the Q4_K_M
// stream for decode and a bf16 copy for the matrix cores).  The fused dequant GEMM
// (kernels/gemm.hip) remains the path when the copies do not fit or AIOS_BLAS=0.
#pragma once
#include <map>
#include <tuple>

#include "common.h"

namespace aios {

class BlasGemm {
 public:
  BlasGemm();
  ~BlasGemm();
  bool ok() const { return ok_; }
  // C[M][ldc] (fp32) = A[M][lda] (bf16) x W[N][ldw]^T (bf16) + beta * C
  void gemm(const bf16_t* A, int lda, const bf16_t* W, int ldw, float* C, int ldc, int M, int N, int K, float beta,
            hipStream_t st);

 private:
  struct Plan;
  Plan* plan(int M, int N, int K, int lda, int ldw, int ldc, bool beta);
  void* handle_ = nullptr;
  void* workspace_ = nullptr;
  size_t ws_bytes_ = 64ull << 20;
  bool ok_ = false;
  std::map<std::tuple<int, int, int, int, int, int, int>, Plan*> plans_;
};

}  // namespace aios
