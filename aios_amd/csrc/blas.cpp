// hipBLASLt bf16 TN GEMM with fp32 output for long prefill chunks (see blas.h).
//
// Row-major C[M][N] = A[M][K] . W[N][K]^T is, in hipBLASLt's column-major terms, the N x M matrix
// C^T = op_T(W^T) . A^T: W (K contiguous per row) is a K x N column-major matrix taken transposed,
// the activations a K x M column-major matrix taken as is -- the "TN" layout the library tunes
// best.  One plan (descriptors + the heuristic's first algorithm) per (M, N, K, lda, ldc).
#include "blas.h"

#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>

namespace aios {

struct BlasGemm::Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};

static bool lt_ok(hipblasStatus_t s) { return s == HIPBLAS_STATUS_SUCCESS; }

BlasGemm::BlasGemm(size_t workspace_bytes) {
  hipblasLtHandle_t h = nullptr;
  if (!lt_ok(hipblasLtCreate(&h))) return;
  if (hipMalloc(&ws_, workspace_bytes) != hipSuccess) {
    hipblasLtDestroy(h);
    ws_ = nullptr;
    return;
  }
  ws_bytes_ = workspace_bytes;
  handle_ = h;
}

BlasGemm::~BlasGemm() {
  for (auto& kv : plans_) {
    Plan* p = kv.second;
    if (p->desc) hipblasLtMatmulDescDestroy(p->desc);
    if (p->a) hipblasLtMatrixLayoutDestroy(p->a);
    if (p->b) hipblasLtMatrixLayoutDestroy(p->b);
    if (p->c) hipblasLtMatrixLayoutDestroy(p->c);
    delete p;
  }
  if (ws_) (void)hipFree(ws_);
  if (handle_) hipblasLtDestroy((hipblasLtHandle_t)handle_);
}

BlasGemm::Plan* BlasGemm::plan(int M, int N, int K, int lda, int ldc) {
  const auto key = std::make_tuple(M, N, K, lda, ldc);
  auto it = plans_.find(key);
  if (it != plans_.end()) return it->second;
  Plan* p = new Plan();
  plans_[key] = p;
  bool ok = lt_ok(hipblasLtMatmulDescCreate(&p->desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  ok = ok && lt_ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  ok = ok && lt_ok(hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  // A operand = the weights: K x N column-major (ld K); B = the activations: K x M (ld lda);
  // C = D: N x M fp32 (ld ldc)
  ok = ok && lt_ok(hipblasLtMatrixLayoutCreate(&p->a, HIP_R_16BF, K, N, K));
  ok = ok && lt_ok(hipblasLtMatrixLayoutCreate(&p->b, HIP_R_16BF, K, M, lda));
  ok = ok && lt_ok(hipblasLtMatrixLayoutCreate(&p->c, HIP_R_32F, N, M, ldc));
  hipblasLtMatmulPreference_t pref = nullptr;
  ok = ok && lt_ok(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = ws_bytes_;
  ok = ok && lt_ok(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                         sizeof(wsb)));
  if (ok) {
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    ok = lt_ok(hipblasLtMatmulAlgoGetHeuristic((hipblasLtHandle_t)handle_, p->desc, p->a, p->b, p->c, p->c, pref, 1,
                                               res, &n)) &&
         n > 0 && lt_ok(res[0].state);
    if (ok) {
      p->algo = res[0].algo;
      p->ws = res[0].workspaceSize;
      ok = p->ws <= ws_bytes_;
    }
  }
  if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  p->ok = ok;
  if (!ok && std::getenv("AIOS_TRACE"))
    std::fprintf(stderr, "[aios] hipBLASLt: no algorithm for M=%d N=%d K=%d (own GEMM used)\n", M, N, K);
  return p;
}

bool BlasGemm::gemm(const bf16_t* A, int lda, const bf16_t* W, float* C, int ldc, int M, int N, int K,
                    bool accumulate, hipStream_t st) {
  if (!handle_ || M <= 0) return false;
  Plan* p = plan(M, N, K, lda, ldc);
  if (!p->ok) return false;
  const float alpha = 1.f, beta = accumulate ? 1.f : 0.f;
  return lt_ok(hipblasLtMatmul((hipblasLtHandle_t)handle_, p->desc, &alpha, W, p->a, A, p->b, &beta, C, p->c, C, p->c,
                               &p->algo, ws_, p->ws, st));
}

}  // namespace aios
