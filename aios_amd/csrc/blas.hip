// hipBLASLt bf16 x bf16 -> fp32 GEMM with cached heuristic plans (see blas.h).
//
// Row-major C[M][N] = A[M][K] . W[N][K]^T is, in hipBLASLt's column-major terms,
// C^T (N x M, ld = ldc) = op_T(W^T stored K x N, ld = ldw) . (A^T stored K x M, ld = lda).
#include "blas.h"

#include <hipblaslt/hipblaslt.h>

#include <stdexcept>
#include <string>

namespace aios {

#define BLAS_CHECK(expr)                                                                          \
  do {                                                                                            \
    hipblasStatus_t s_ = (expr);                                                                  \
    if (s_ != HIPBLAS_STATUS_SUCCESS)                                                             \
      throw std::runtime_error(std::string("hipBLASLt: ") + #expr + " failed (" + std::to_string((int)s_) + ")"); \
  } while (0)

struct BlasGemm::Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool has_algo = false;
};

BlasGemm::BlasGemm() {
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return;
  handle_ = h;
  if (hipMalloc(&workspace_, ws_bytes_) != hipSuccess) {
    workspace_ = nullptr;
    ws_bytes_ = 0;
  }
  ok_ = true;
}

BlasGemm::~BlasGemm() {
  for (auto& kv : plans_) {
    Plan* p = kv.second;
    if (p->desc) hipblasLtMatmulDescDestroy(p->desc);
    if (p->la) hipblasLtMatrixLayoutDestroy(p->la);
    if (p->lb) hipblasLtMatrixLayoutDestroy(p->lb);
    if (p->lc) hipblasLtMatrixLayoutDestroy(p->lc);
    delete p;
  }
  if (workspace_) hipFree(workspace_);
  if (handle_) hipblasLtDestroy((hipblasLtHandle_t)handle_);
}

BlasGemm::Plan* BlasGemm::plan(int M, int N, int K, int lda, int ldw, int ldc, bool beta) {
  const auto key = std::make_tuple(M, N, K, lda, ldw, ldc, (int)beta);
  auto it = plans_.find(key);
  if (it != plans_.end()) return it->second;
  Plan* p = new Plan();
  BLAS_CHECK(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  BLAS_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  BLAS_CHECK(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  BLAS_CHECK(hipblasLtMatrixLayoutCreate(&p->la, HIP_R_16BF, K, N, ldw));  // W^T stored K x N
  BLAS_CHECK(hipblasLtMatrixLayoutCreate(&p->lb, HIP_R_16BF, K, M, lda));  // A^T stored K x M
  BLAS_CHECK(hipblasLtMatrixLayoutCreate(&p->lc, HIP_R_32F, N, M, ldc));   // C^T N x M
  hipblasLtMatmulPreference_t pref = nullptr;
  BLAS_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = ws_bytes_;
  BLAS_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[4];
  int n = 0;
  hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic((hipblasLtHandle_t)handle_, p->desc, p->la, p->lb, p->lc,
                                                      p->lc, pref, 4, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (s == HIPBLAS_STATUS_SUCCESS && n > 0) {
    p->algo = res[0].algo;
    p->has_algo = true;
  }
  (void)beta;
  plans_[key] = p;
  return p;
}

void BlasGemm::gemm(const bf16_t* A, int lda, const bf16_t* W, int ldw, float* C, int ldc, int M, int N, int K,
                    float beta, hipStream_t st) {
  if (!ok_) throw std::runtime_error("hipBLASLt unavailable");
  Plan* p = plan(M, N, K, lda, ldw, ldc, beta != 0.f);
  const float alpha = 1.f;
  BLAS_CHECK(hipblasLtMatmul((hipblasLtHandle_t)handle_, p->desc, &alpha, W, p->la, A, p->lb, &beta, C, p->lc, C,
                             p->lc, p->has_algo ? &p->algo : nullptr, workspace_, ws_bytes_, st));
}

}  // namespace aios
